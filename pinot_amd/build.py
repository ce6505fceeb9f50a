"""Builds the in-tree HIP extension libpinot_amd.so for gfx950 (hipcc cross-compiles without a GPU).

Incremental: one object per source under csrc/ (kept next to it), rebuilt when the source or a header it includes
(recursively, "..." includes only) is newer than the object; then one link."""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libpinot_amd.so")
SOURCES = ["pa_scan_part_a.hip", "pa_scan_part_b.hip", "pa_scan_part_mv.hip", "pa_scan_std.hip", "pa_scan_lane.hip",
           "pa_scan_gdense.hip", "pa_kernels.hip", "pa_merge.hip", "pa_stats.hip", "pa_pve.hip", "pa_segment.hip",
           "pa_plan.hip", "pa_plan_kernels.hip", "pa_jit.hip", "pa_capi.hip", "pa_fetch.hip", "pa_stats_host.hip"]
# every header under csrc/ (globbed, so a new one is covered without an edit here) and the public C-ABI header
HEADERS = sorted(f for f in os.listdir(CSRC) if f.endswith(".h")) + [os.path.join("..", "..", "include", "pinot_amd.h")]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-munsafe-fp-atomics", "-std=c++17",
         "-Wall", "-Wno-unused-function"]
# kernels compiled at query prepare by hiprtc (pa_jit.hip): their sources become string literals (*_src.inc), with the
# descriptor header they share with the host pasted in
JIT_SOURCES = ["gdl_jit.hip", "pve_jit.hip"]
JIT_ABI = "pa_jit_abi.h"
_INCLUDE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(path, seen=None):
    """path and every "..." include it reaches (resolved next to the including file, then in csrc/ and include/)."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    for inc in _INCLUDE.findall(open(path, errors="replace").read()):
        for d in (os.path.dirname(path), CSRC, os.path.join(HERE, "..", "include")):
            cand = os.path.normpath(os.path.join(d, inc))
            if os.path.exists(cand):
                _deps(cand, seen)
                break
    return seen


def _obj(src):
    return os.path.join(CSRC, os.path.splitext(src)[0] + ".o")


def _stale_objs():
    out = []
    for src in SOURCES:
        o = _obj(src)
        if not os.path.exists(o):
            out.append(src)
            continue
        t = os.path.getmtime(o)
        if any(os.path.getmtime(d) > t for d in _deps(os.path.join(CSRC, src)) | {__file__}):
            out.append(src)
    return out


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS + JIT_SOURCES] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


def jit_source_text(name):
    """A JIT kernel's source with the shared descriptor header pasted in place of its #include line."""
    src = open(os.path.join(CSRC, name)).read()
    abi = open(os.path.join(CSRC, JIT_ABI)).read().replace("#pragma once\n", "")
    inc = '#include "%s"' % JIT_ABI
    if inc in src:
        src = src.replace(inc, abi, 1)
    assert '#include "' not in src, "%s: hiprtc sees no include path" % name
    return src


def _jit_source():
    """The JIT kernels' sources as C++ raw string literals (pa_jit.hip compiles them at query prepare with hiprtc)."""
    for name in JIT_SOURCES:
        src = jit_source_text(name)
        assert ")JITSRC" not in src
        out = os.path.join(CSRC, name.replace(".hip", "_src.inc"))
        text = 'R"JITSRC(' + src + ')JITSRC"\n'
        if not os.path.exists(out) or open(out).read() != text:
            with open(out, "w") as f:
                f.write(text)


def build(force=False, verbose=False):
    if not force and not _stale():
        return LIB
    _jit_source()
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    # one object per stale source, compiled in parallel (each translation unit holds its own kernels), then one link
    todo = SOURCES if force else _stale_objs()
    procs = []
    for src in todo:
        cmd = [hipcc] + [f for f in FLAGS if f != "-shared"] + ["-c", os.path.join(CSRC, src), "-o", _obj(src) + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd)))
    failed = [src for src, p in procs if p.wait() != 0]
    for src, _ in procs:
        if src not in failed:
            os.replace(_obj(src) + ".tmp", _obj(src))
    if failed:
        raise RuntimeError("hipcc failed: %s" % ", ".join(failed))
    cmd = [hipcc] + FLAGS + [_obj(s) for s in SOURCES] + ["-lhiprtc", "-o", LIB + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
