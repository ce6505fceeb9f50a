"""Test-only restatement of the two local halves of parallel.merge_hashed_sections (what the library's pack / merge
kernels in pinot_amd/csrc/pa_merge.hip do on the GPU), in torch tensor ops over a block's section views, so the
exchange protocol runs in multi-process gloo tests on CPU tensors. Not used by the product path (HashedAccumulators
always passes parallel.LibraryRows)."""
import torch
import torch.distributed as dist

from pinot_amd import _lib as L
from pinot_amd.parallel import SECTION_IDENTITY, SECTION_OP, key_owner, key_owner2

_SCATTER_REDUCE = {dist.ReduceOp.SUM: "sum", dist.ReduceOp.MIN: "amin", dist.ReduceOp.MAX: "amax"}


class TorchRows:
    """pack: occupied slots (count > 0) -> byte rows (per-key sections concatenated) grouped by key_owner; merge: rows
    -> the block by packed key (torch.unique + one scatter-reduce per section), slots [0, groups) in ascending key
    order, every other slot empty."""

    def __init__(self, views, num_slots):
        self.views, self.num_slots = views, num_slots
        self.per_key = [(k, t) for k, t in views if k != L.PA_ACC_DOCS_U64]

    def pack(self, world):
        ns = self.num_slots
        count = dict(self.per_key)[L.PA_ACC_COUNT_U64]
        occ = torch.nonzero(count.view(ns) > 0).flatten()
        m = int(occ.numel())
        parts = []
        self.layout = []
        for k, t in self.per_key:
            w = t.numel() // ns
            b = t.view(ns, w)[occ].contiguous().view(torch.uint8).view(m, -1) if m else \
                torch.empty(0, w * t.element_size(), dtype=torch.uint8)
            self.layout.append((k, t.dtype, w, b.shape[1]))
            parts.append(b)
        local = torch.cat(parts, dim=1)
        kt = dict(self.per_key)[L.PA_ACC_KEYS_I64]
        kw = kt.numel() // ns  # 1, or 3 for two-word keys: [k0, k1, state]
        keys = kt.view(ns, kw)[occ]
        owner = key_owner(keys[:, 0], world) if kw == 1 else key_owner2(keys[:, 0], keys[:, 1], world)
        order = torch.argsort(owner, stable=True)
        return local[order], torch.bincount(owner, minlength=world).tolist()

    def merge(self, rows):
        ns = self.num_slots
        cols, o = {}, 0
        for k, dt, w, nb in self.layout:
            cols[k] = rows[:, o:o + nb].contiguous().view(dt).view(-1, w)
            o += nb
        kc = cols[L.PA_ACC_KEYS_I64]
        kw = kc.shape[1]
        uniq, inv = torch.unique(kc[:, 0] if kw == 1 else kc[:, :2], dim=None if kw == 1 else 0, sorted=True,
                                 return_inverse=True)
        u = int(uniq.shape[0])
        if u > ns:
            return u, u - ns
        for k, t in self.per_key:
            w = t.numel() // ns
            out = t.view(ns, w)
            out.fill_(SECTION_IDENTITY.get(k, 0))
            if k == L.PA_ACC_KEYS_I64:
                if w == 1:
                    out[:u, 0] = uniq
                else:
                    out[:u, :2] = uniq
                    out[:u, 2] = 0  # (a state other than empty)
                continue
            acc = torch.full((u, w), SECTION_IDENTITY.get(k, 0), dtype=t.dtype)
            acc.scatter_reduce_(0, inv.view(-1, 1).expand(-1, w), cols[k], reduce=_SCATTER_REDUCE[SECTION_OP[k]],
                                include_self=True)
            out[:u] = acc
        return u, 0
