"""Builds the in-tree HIP extension libpinot_amd.so for gfx950 (hipcc cross-compiles without a GPU)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libpinot_amd.so")
SOURCES = ["pa_scan_part_a.hip", "pa_scan_part_b.hip", "pa_scan_part_mv.hip", "pa_scan_std.hip", "pa_scan_lane.hip", "pa_scan_gdense.hip", "pa_kernels.hip", "pa_merge.hip", "pa_stats.hip", "pa_pve.hip", "pa_capi.hip"]
# every header under csrc/ (globbed, so a new one is covered without an edit here) and the public C-ABI header
HEADERS = sorted(f for f in os.listdir(CSRC) if f.endswith(".h")) + [os.path.join("..", "..", "include", "pinot_amd.h")]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-munsafe-fp-atomics", "-std=c++17",
         "-Wall", "-Wno-unused-function"]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS + JIT_SOURCES] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


JIT_SOURCES = ["gdl_jit.hip", "pve_jit.hip"]


def _jit_source():
    """The JIT kernels' sources as C++ raw string literals (pa_capi.hip compiles them at query prepare with hiprtc)."""
    for name in JIT_SOURCES:
        src = open(os.path.join(CSRC, name)).read()
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
    # one object per source, compiled in parallel (each translation unit holds its own kernels), then one link
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc] + [f for f in FLAGS if f != "-shared"] + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    if any(p.wait() != 0 for p in procs):
        raise RuntimeError("hipcc failed")
    cmd = [hipcc] + FLAGS + objs + ["-lhiprtc", "-o", LIB + ".tmp"]
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
