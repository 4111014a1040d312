"""Multi-GPU analysis: one process per GPU, buffers sharded, counters merged
with RCCL (torch.distributed "nccl") over xGMI.

The reference analyses the `samples` list on one thread
(src/mem_sampling.c:324-342); each buffer is independent given the read-only
object table (__analyze_buffer only reads samples->thread_rank/access_type and
the table), so the analysis-ordered buffer list is split into contiguous,
byte-balanced ranges, one per rank.  Every rank carries its range's global
analysis index (seq_base) so first-match ordinals stay globally comparable.
The only exchange step is the merge of the counters:

* u64 sums (global counts/weights, per-object counts/weights/levels)  -> SUM
* u64 mins (global bucket min_weight, first-match ordinals, error word) -> MIN
* u64 maxes (global bucket max_weight)                                 -> MAX
* u32 page histogram                                                   -> SUM
  (packed, merge_hist_packed: bytes of the cells <= 255 / world summed as
  u8, the larger cells gathered as (cell, count) lists -- 98 -> ~26 MB per
  rank at 1M intervals)
* sparse page cells, per-buffer counts: variable length -> gathered to the root

RCCL reduces int64, not uint64: sums are bit-identical under two's
complement; MIN/MAX use the order-preserving map x ^ 2^63.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

INT64_MIN = -(1 << 63)


def shard_ranges(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) buffer ranges with balanced byte counts."""
    lengths = np.asarray(lengths, dtype=np.int64)
    n = lengths.shape[0]
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    csum = np.concatenate([[0], np.cumsum(lengths)])
    total = csum[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        c = int(np.searchsorted(csum, target, side="left"))
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def _collective(t, rop, dst, group):
    """reduce / all_reduce; a device tensor goes through host memory when the
    backend is not RCCL (gloo test runs)."""
    import torch.distributed as dist

    staged = t.is_cuda and dist.get_backend(group) != "nccl"
    x = t.cpu() if staged else t
    if dst is None:
        dist.all_reduce(x, op=rop, group=group)
    else:
        dist.reduce(x, dst=dst, op=rop, group=group)
    if staged:
        t.copy_(x)
    return t


def reduce_u64(t, op: str, dst: Optional[int] = 0, group=None):
    """Reduce a tensor of u64 bit patterns stored as int64.  dst=None -> all-reduce."""
    import torch
    import torch.distributed as dist

    assert t.dtype == torch.int64
    flip = op in ("min", "max")
    if flip:
        t.bitwise_xor_(INT64_MIN)
    rop = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op]
    _collective(t, rop, dst, group)
    if flip:
        t.bitwise_xor_(INT64_MIN)
    return t


def reduce_u32_sum(t, dst: Optional[int] = 0, group=None):
    import torch
    import torch.distributed as dist

    assert t.dtype == torch.int32
    return _collective(t, dist.ReduceOp.SUM, dst, group)


class HistPacker:
    """Buffers of the packed page-histogram merge of one engine (allocated
    once; the overflow list holds up to `ovf_frac` of the cells)."""

    def __init__(self, eng, device, ovf_frac: float = 0.125):
        import torch

        from . import _lib

        self.eng = eng
        self.cells = eng.array_size(_lib.NMG_ARR_HIST32)
        self.cap = max(1024, int(self.cells * ovf_frac))
        self.u8 = torch.empty(max(self.cells, 4), dtype=torch.uint8, device=device)
        # (empty, not zeros: a fill on torch's stream is not ordered with
        # nmg_hist_pack, which writes entries [0, n) on the engine's own
        # non-blocking stream; merge() zeroes the padding [n, nmax) itself)
        self.ovf = torch.empty(self.cap, dtype=torch.int64, device=device)
        self.n = torch.zeros(1, dtype=torch.int64, device=device)
        self.dense = None  # fallback: the u32 histogram (a list longer than cap)

    def merge(self, dst: int = 0, group=None) -> int:
        """Merge every rank's histogram into rank dst's engine; returns the
        bytes this rank contributed to the collectives."""
        import torch
        import torch.distributed as dist

        from . import _lib

        if not self.cells:
            return 0
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        thr = 255 // world
        n = self.eng.hist_pack(thr, self.u8.data_ptr(), self.ovf.data_ptr(), self.cap)
        self.n.fill_(n)
        _collective(self.n, dist.ReduceOp.MAX, None, group)  # every rank: the longest list
        nmax = int(self.n.item())
        if nmax > self.cap:  # some list does not fit: the plain u32 reduce
            if self.dense is None:
                self.dense = torch.empty(self.cells, dtype=torch.int32, device=self.u8.device)
            self.eng.export_array(_lib.NMG_ARR_HIST32, self.dense.data_ptr())
            reduce_u32_sum(self.dense, dst=dst, group=group)
            if rank == dst:
                torch.cuda.synchronize(self.u8.device)
                self.eng.import_array(_lib.NMG_ARR_HIST32, self.dense.data_ptr())
            return self.cells * 4
        if n < nmax:
            self.ovf[n:nmax].zero_()  # (padding: count 0)
        _collective(self.u8[:self.cells], dist.ReduceOp.SUM, dst, group)
        part = self.ovf[:nmax]
        if dist.get_backend(group) == "nccl":
            out = [torch.empty_like(part) for _ in range(world)] if rank == dst else None
            dist.gather(part, out, dst=dst, group=group)
        else:  # (gloo test runs: host staging)
            cpu = part.cpu()
            out = [torch.empty_like(cpu) for _ in range(world)] if rank == dst else None
            dist.gather(cpu, out, dst=dst, group=group)
        if rank == dst:
            allovf = torch.cat([o.to(self.u8.device) for o in out]) if nmax else self.ovf[:0]
            torch.cuda.synchronize(self.u8.device)
            self.eng.hist_unpack(self.u8.data_ptr(), allovf.data_ptr() if nmax else 0, allovf.numel())
        return self.cells + nmax * 8


GLOBAL_SUM_WORDS = 2 * 39  # sum64's head: [2 access][39] global sums (nmg_internal.h kGlobalSums)
LEVEL_WORDS = 37           # per entry and access: na, 18 x (count, sum) (nmg_internal.h kLevelWords)
GLOBAL_MIN_WORDS = 2 * 18  # min64's head: [2][18] bucket minima, then [E] ordinals and the error word


class ObjPacker:
    """Buffers of the packed per-object counter merge of one engine
    (nmg_objcw_pack / nmg_objcw_unpack): sum64's four count / weight rows as
    u32 words -- a value below 2^32 / world, so that the sum over the ranks
    fits -- plus a list of the larger values as (row word, value) pairs
    (allocated once; the list holds up to `ovf_frac` of the words)."""

    def __init__(self, eng, device, ovf_frac: float = 1 / 64):
        import torch

        from . import _lib

        self.eng = eng
        n = eng.array_size(_lib.NMG_ARR_SUM64)
        levels = bool(eng.flags & _lib.NMG_F_OBJECT_LEVELS)
        per = 4 + (2 * LEVEL_WORDS if levels else 0)  # (levels: [E][2][37] after the rows)
        # the entry count from min64 ([2][18] minima, [E] ordinals, error word), checked
        # against sum64's size: a layout change in nmg_internal.h fails here, not silently
        self.E = eng.array_size(_lib.NMG_ARR_MIN64) - GLOBAL_MIN_WORDS - 1 if n else 0
        if n and self.E * per + GLOBAL_SUM_WORDS != n:
            raise RuntimeError(f"ObjPacker: sum64 holds {n} words, not {GLOBAL_SUM_WORDS} + {per} x {self.E} entries")
        self.n_sum64 = n  # the engine's sum64 size this packer was built for
        self.levels = levels
        self.rows = 4 * self.E
        self.cap = max(1024, int(self.rows * ovf_frac))
        self.u32 = torch.empty(max(self.rows, 1), dtype=torch.int32, device=device)
        self.ovf = torch.empty(2 * self.cap, dtype=torch.int64, device=device)
        self.n = torch.zeros(1, dtype=torch.int64, device=device)

    def merge(self, t, dst: int = 0, group=None):
        """The rows of the sum64 image t (every rank's) summed into rank dst's
        t; returns the bytes this rank contributed, or None when some rank's
        list outgrew its buffer (the caller reduces the rows as u64)."""
        import torch
        import torch.distributed as dist

        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        thr = (1 << 32) // world
        n = self.eng.objcw_pack(t.data_ptr(), thr, self.u32.data_ptr(), self.ovf.data_ptr(), self.cap)
        self.n.fill_(n)
        _collective(self.n, dist.ReduceOp.MAX, None, group)
        nmax = int(self.n.item())
        if nmax > self.cap:
            return None
        if n < nmax:
            self.ovf[2 * n:2 * nmax].zero_()  # (padding: row word 0 += 0)
        _collective(self.u32[:self.rows], dist.ReduceOp.SUM, dst, group)  # (u32 sums as int32: the same bits)
        part = self.ovf[:2 * nmax]
        if dist.get_backend(group) == "nccl":
            out = [torch.empty_like(part) for _ in range(world)] if rank == dst else None
            dist.gather(part, out, dst=dst, group=group)
        else:  # (gloo test runs: host staging)
            cpu = part.cpu()
            out = [torch.empty_like(cpu) for _ in range(world)] if rank == dst else None
            dist.gather(cpu, out, dst=dst, group=group)
        if rank == dst:
            allovf = torch.cat([o.to(self.u32.device) for o in out]) if nmax else self.ovf[:0]
            torch.cuda.synchronize(self.u32.device)
            self.eng.objcw_unpack(t.data_ptr(), self.u32.data_ptr(), allovf.data_ptr() if nmax else 0,
                                  allovf.numel() // 2)
        return self.rows * 4 + nmax * 16


def gather_arrays(a: np.ndarray, dst: int = 0, group=None):
    """Variable-length gather of a numpy array; returns the list on dst."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    out = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(a, out, dst=dst, group=group)
    return out


def merge_sparse(parts) -> Tuple[np.ndarray, np.ndarray]:
    keys = np.concatenate([p[0] for p in parts]) if parts else np.zeros(0, np.uint64)
    vals = np.concatenate([p[1] for p in parts]) if parts else np.zeros(0, np.uint32)
    if keys.shape[0] == 0:
        return keys.astype(np.uint64), vals.astype(np.uint32)
    u, inv = np.unique(keys, return_inverse=True)
    s = np.zeros(u.shape[0], dtype=np.uint64)
    np.add.at(s, inv, vals.astype(np.uint64))
    return u, (s & 0xFFFFFFFF).astype(np.uint32)


def merge_engine(eng, dst: int = 0, group=None, device=None, packed_hist: bool = False) -> int:
    """Merge every rank's partial counters into rank dst's engine (RCCL reduce
    of the dense arrays over xGMI; gathers of the small variable-length ones).
    packed_hist: the page histogram through HistPacker (bytes + overflow)
    and the per-object counters through ObjPacker (u32 words + overflow).
    Returns the bytes this rank contributed to the dense collectives."""
    import torch
    import torch.distributed as dist

    from . import _lib

    rank = dist.get_rank(group)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    nbytes = 0
    for which, op in ((_lib.NMG_ARR_SUM64, "sum"), (_lib.NMG_ARR_MIN64, "min"), (_lib.NMG_ARR_MAX64, "max")):
        n = eng.array_size(which)
        if n == 0:
            continue
        t = torch.empty(n, dtype=torch.int64, device=dev)
        eng.export_array(which, t.data_ptr())
        got = None
        if packed_hist and which == _lib.NMG_ARR_SUM64:  # the per-object rows as u32 + a list
            op_ = getattr(eng, "_obj_packer", None)  # rebuilt whenever the table's size changed
            if op_ is None or op_.n_sum64 != n or op_.levels != bool(eng.flags & _lib.NMG_F_OBJECT_LEVELS):
                op_ = eng._obj_packer = ObjPacker(eng, dev)
            got = op_.merge(t, dst=dst, group=group)
            if got is not None:
                nbytes += got
                rest = [t[:GLOBAL_SUM_WORDS]] + ([t[GLOBAL_SUM_WORDS + op_.rows:]] if n > GLOBAL_SUM_WORDS + op_.rows else [])
                for part in rest:  # the global sums (and per-object levels) as u64
                    nbytes += 8 * part.numel()
                    reduce_u64(part, "sum", dst=dst, group=group)
        if got is None:
            nbytes += 8 * n
            reduce_u64(t, op, dst=dst, group=group)
        if rank == dst:
            torch.cuda.synchronize(dev)
            eng.import_array(which, t.data_ptr())
    n = eng.array_size(_lib.NMG_ARR_HIST32)
    if n and packed_hist:
        hp = getattr(eng, "_hist_packer", None)  # one packer per engine, reused across merges
        if hp is None or hp.cells != n:
            hp = eng._hist_packer = HistPacker(eng, dev)
        nbytes += hp.merge(dst=dst, group=group)
    elif n:
        nbytes += 4 * n
        t = torch.empty(n, dtype=torch.int32, device=dev)
        eng.export_array(_lib.NMG_ARR_HIST32, t.data_ptr())
        reduce_u32_sum(t, dst=dst, group=group)
        if rank == dst:
            torch.cuda.synchronize(dev)
            eng.import_array(_lib.NMG_ARR_HIST32, t.data_ptr())
    merge_host_side(eng, dst=dst, group=group)
    return nbytes


def merge_host_side(eng, dst: int = 0, group=None) -> None:
    """Sparse page cells and per-buffer counts (variable length): gathered."""
    import torch.distributed as dist

    rank = dist.get_rank(group)
    k, v = eng.sparse_export()
    parts = gather_arrays(np.stack([k, v.astype(np.uint64)]) if k.shape[0] else np.zeros((2, 0), np.uint64),
                          dst=dst, group=group)
    s, f = eng.buffer_counts()
    nbytes = np.asarray(eng.buffer_bytes, dtype=np.uint64)
    counts = gather_arrays(np.stack([s.astype(np.uint64), f.astype(np.uint64), nbytes]), dst=dst, group=group)
    if rank == dst:
        keys, vals = merge_sparse([(p[0], p[1].astype(np.uint32)) for p in parts])
        eng.sparse_import(keys, vals)
        allc = np.concatenate(counts, axis=1)
        eng.set_buffer_counts(allc[0].astype(np.uint32), allc[1].astype(np.uint32), allc[2])
