"""Multi-GPU sharding of the exhaustive scans.

One process per GPU (torchrun / torch.distributed.run).  Pairs are independent units once
every rank holds the genotype panel, P and Py, so the scan shards with no collective on
its hot path:

* genotype panel: each rank reads (or generates) its contiguous shard of SNPs and the
  packed 2-bit shards are all-gathered -- RCCL over xGMI with the ``nccl`` backend
  (25 MB at 2,000 x 50,000), gloo on CPU;
* P and Py: computed on rank 0 and broadcast (32 MB at n = 2,000);
* scan: rank r scans the rows of part r+1 of the reference's triangle-folded split
  ``parallel=[N, r+1]`` (remma_epiAA.py:125-139), equal pair counts per rank;
* hits: gathered to rank 0 and merged in (i, j) order -- the same rows and order a
  single-GPU scan writes, bit-identical values (each pair is computed by one rank with a
  fixed reduction order).

The per-rank compute is injected (``scan_fn``) so the sharding and merge logic is tested
on CPU with gloo and the oracle; the product path passes the HIP plan's scan.
"""
import os

import numpy as np


def world():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend=None):
    """Initialise torch.distributed when WORLD_SIZE > 1.  Returns the backend used (None
    for a single process).  ``nccl`` is RCCL on ROCm."""
    rank, ws, local = world()
    if ws <= 1:
        return None
    import torch
    import torch.distributed as dist
    if dist.is_initialized():
        return dist.get_backend()
    if backend is None:
        backend = os.environ.get("GMAT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return backend


def _device(backend):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def allreduce_max(x):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device(dist.get_backend()))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(x):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device(dist.get_backend()))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def snp_shard(m, rank, ws):
    """Contiguous SNP range [lo, hi) owned by `rank` for loading."""
    per = (m + ws - 1) // ws
    return min(m, rank * per), min(m, (rank + 1) * per)


def allgather_packed(local_rows, m, nb):
    """All-gather the packed .bed rows (uint8, (hi-lo) x nb) of every rank's SNP shard into
    the full (m x nb) packed panel (RCCL all_gather on the GPU with nccl)."""
    import torch
    import torch.distributed as dist
    rank, ws, _ = world()
    if not (dist.is_available() and dist.is_initialized()) or ws == 1:
        return np.ascontiguousarray(local_rows).reshape(-1)
    per = (m + ws - 1) // ws
    dev = _device(dist.get_backend())
    buf = np.zeros((per, nb), dtype=np.uint8)
    buf[: local_rows.shape[0]] = local_rows
    src = torch.from_numpy(buf).to(dev)
    outs = [torch.empty_like(src) for _ in range(ws)]
    dist.all_gather(outs, src)
    full = torch.cat(outs, dim=0)[:m].cpu().numpy()
    return np.ascontiguousarray(full).reshape(-1)


def broadcast_array(arr, src=0, shape=None, dtype=np.float64):
    """Broadcast a numpy array from `src` (other ranks pass arr=None with shape)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return arr
    dev = _device(dist.get_backend())
    if dist.get_rank() == src:
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=dtype)).to(dev)
    else:
        t = torch.empty(tuple(shape), dtype=torch.from_numpy(np.zeros(1, dtype)).dtype, device=dev)
    dist.broadcast(t, src)
    return t.cpu().numpy()


def rank_rows(kind, num_snp, rank, ws, rows=None):
    """Rows this rank scans: part rank+1 of the reference's folded split, restricted to
    `rows` when the caller scans a subset."""
    from .remma._scan import parallel_rows
    mine = np.array(sorted(parallel_rows(num_snp, [ws, rank + 1], kind)), dtype=np.int64)
    if rows is not None:
        mine = np.intersect1d(mine, np.asarray(rows, dtype=np.int64))
    return mine


def merge_hits(parts):
    """Concatenate per-rank hit tuples (i, j, eff, var, chi, p) and sort by (i, j)."""
    parts = [p for p in parts if p is not None and len(p[0])]
    if not parts:
        return tuple(np.zeros(0, np.int64) if t < 2 else np.zeros(0) for t in range(6))
    cat = [np.concatenate([p[t] for p in parts]) for t in range(6)]
    order = np.lexsort((cat[1], cat[0]))
    return tuple(c[order] for c in cat)


def distributed_scan(scan_fn, kind, num_snp, p_cut, rows=None):
    """Run ``scan_fn(kind, my_rows, p_cut) -> (i, j, eff, var, chi, p)`` on this rank's
    share and gather the merged hits on rank 0 (other ranks get None)."""
    rank, ws, _ = world()
    if ws > 1:
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("WORLD_SIZE=%d but no process group is initialised: a single rank would "
                               "return only its own share of the hits (call dist.init() first)" % ws)
    mine = rank_rows(kind, num_snp, rank, ws, rows)
    local = scan_fn(kind, mine, p_cut) if mine.size else None
    if ws == 1:
        return merge_hits([local])
    gathered = [None] * ws if rank == 0 else None
    dist.gather_object(None if local is None else tuple(np.asarray(a) for a in local), gathered, dst=0)
    return merge_hits(gathered) if rank == 0 else None
