"""Multi-GPU sharding of the exhaustive scans.

One process per GPU (launched by torch.distributed.run / torchrun, which only sets RANK,
WORLD_SIZE, LOCAL_RANK, MASTER_*).  Pairs are independent units once every rank holds the
genotype panel, P and Py, so the scan shards with no collective on its hot path:

* genotype panel: each rank reads (or generates) its contiguous shard of SNPs and the packed
  2-bit shards are all-gathered (25 MB at 2,000 x 50,000);
* P and Py: computed on rank 0 and broadcast (32 MB at n = 2,000);
* scan plan: its spectral state (eigendecomposition, certificates, low-rank basis) computed on
  rank 0 and broadcast (shared_plan), the slices and codings built locally;
* scan: rank r scans the rows of part r+1 of the reference's triangle-folded split
  ``parallel=[N, r+1]`` (remma_epiAA.py:125-139), equal pair counts per rank;
* hits: gathered to rank 0 and merged in (i, j) order -- the same rows and order a
  single-GPU scan writes, bit-identical values (each pair is computed by one rank with a
  fixed reduction order).

Backends.  ``rccl`` (the product path on GPUs): the exchanges run in libgmat_hip on RCCL over
xGMI (gmat_comm_* in include/gmat_hip.h); no PyTorch is imported.  The 128-byte unique id is
created by rank 0 and shared through a file in the temp directory keyed by the launcher
(single-node runs, as bench.py's contract): the key holds the launcher's pid AND its start time,
MASTER_PORT, the run id and the restart count, so a file left by a crashed run is never read.
When WORLD_SIZE > 1 and a GPU is visible the backend is RCCL on every rank, and any RCCL failure
raises (the launcher then stops the job) -- there is no silent per-rank fallback that could leave
ranks on different backends.  ``gloo`` (torch.distributed on CPU) is the test harness of
tests/test_dist_cpu.py, chosen only when no GPU is visible or GMAT_DIST_BACKEND=gloo says so.
"""
import ctypes
import os
import tempfile
import time

import numpy as np

_state = {"backend": None, "comm": None}


def world():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def backend():
    return _state["backend"]


def _proc_start(pid):
    """Start time of a process in clock ticks since boot (/proc/<pid>/stat field 22), 0 if unknown."""
    try:
        with open("/proc/%d/stat" % pid) as f:
            return int(f.read().rsplit(")", 1)[1].split()[19])
    except (OSError, ValueError, IndexError):
        return 0


def _id_file():
    """Rendezvous file of this launch: every rank of one torchrun agent computes the same name, and
    no earlier launch can (the agent's pid is paired with its start time)."""
    ppid = os.getppid()
    key = "%s_%s_%s_%d_%d" % (os.environ.get("MASTER_PORT", "0"), os.environ.get("TORCHELASTIC_RUN_ID", "na"),
                              os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"), ppid, _proc_start(ppid))
    return os.path.join(tempfile.gettempdir(), "gmat_rccl_id_" + key)


def _init_rccl(rank, ws):
    from . import _native as N
    lib = N.ensure_device()  # binds LOCAL_RANK's GPU before the communicator
    path = _id_file()
    uid = (ctypes.c_uint8 * 128)()
    if rank == 0:
        N.check(lib.gmat_comm_unique_id(uid), "gmat_comm_unique_id")
        tmp = path + ".tmp%d" % os.getpid()
        with open(tmp, "wb") as f:
            f.write(bytes(uid))
        os.replace(tmp, path)
    else:
        t0 = time.time()
        while True:
            try:
                with open(path, "rb") as f:
                    data = f.read()
                if len(data) == 128:
                    break
            except FileNotFoundError:
                pass
            if time.time() - t0 > 120:
                raise RuntimeError("rank %d: no RCCL unique id from rank 0 at %s" % (rank, path))
            time.sleep(0.01)
        ctypes.memmove(uid, data, 128)
    comm = ctypes.c_void_p()
    N.check(lib.gmat_comm_init(ctypes.byref(comm), ws, rank, uid), "gmat_comm_init")
    _state["comm"] = comm
    N.check(lib.gmat_comm_barrier(comm), "gmat_comm_barrier")
    if rank == 0:
        try:
            os.remove(path)
        except OSError:
            pass


def choose_backend(explicit=None, gpu_visible=None, n_devices=None, world_size=None):
    """The backend every rank uses: GMAT_DIST_BACKEND / the argument when given, else ``rccl``
    when every rank has a GPU of its own (the product path) and ``gloo`` otherwise (the CPU test
    harness, or more ranks than GPUs: RCCL refuses two ranks on one device).  The choice depends
    only on the launch environment, identical on all ranks of a node."""
    if explicit is None:
        explicit = os.environ.get("GMAT_DIST_BACKEND")
    if explicit is not None:
        if explicit not in ("rccl", "gloo"):
            raise ValueError("unknown backend %r (rccl | gloo)" % explicit)
        return explicit
    if gpu_visible is None:
        from . import _native as N
        lib = N.load(required=False)
        n_devices = N.device_count() if lib is not None else 0
        gpu_visible = n_devices > 0
    if world_size is None:
        world_size = world()[1]
    if gpu_visible and n_devices is not None and n_devices < world_size:
        from . import _native as N
        if not N.shared_gpu_allowed():
            raise RuntimeError("%d ranks but %d GPU(s) visible: one process per GPU (GMAT_ALLOW_SHARED_GPU=1 "
                               "lets ranks share devices over gloo, for tests)" % (world_size, n_devices))
        return "gloo"
    return "rccl" if gpu_visible else "gloo"


def init(backend=None):
    """Set up the process group when WORLD_SIZE > 1.  Returns the backend used (None for a
    single process).  RCCL errors are fatal (no fallback: ranks must agree on the backend)."""
    rank, ws, local = world()
    if ws <= 1:
        return None
    if _state["backend"] is not None:
        return _state["backend"]
    backend = choose_backend(backend)
    if backend == "rccl":
        try:
            _init_rccl(rank, ws)
        except Exception as exc:
            raise RuntimeError("rank %d/%d: RCCL communicator setup failed (%s); set GMAT_DIST_BACKEND=gloo to "
                               "exchange over host TCP instead (e.g. several ranks on one GPU)" % (rank, ws, exc))
    if backend == "gloo":
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not tdist.is_initialized():
            tdist.init_process_group("gloo")
            # tear the gloo group down before interpreter shutdown: left to the destructors, its
            # worker threads can be destroyed while joinable (std::terminate, exit status -6)
            import atexit
            atexit.register(_destroy_gloo)
    _state["backend"] = backend
    return backend


def _destroy_gloo():
    import torch.distributed as tdist
    if tdist.is_initialized():
        try:
            tdist.barrier()
        finally:
            tdist.destroy_process_group()


def _require():
    rank, ws, _ = world()
    if ws > 1 and _state["backend"] is None:
        raise RuntimeError("WORLD_SIZE=%d but no process group is initialised: a single rank would "
                           "see only its own share (call dist.init() first)" % ws)
    return _state["backend"]


def _lib():
    from . import _native as N
    return N, N.load()


def barrier():
    b = _require()
    if b == "rccl":
        N, lib = _lib()
        N.check(lib.gmat_comm_barrier(_state["comm"]), "gmat_comm_barrier")
    elif b == "gloo":
        import torch.distributed as tdist
        tdist.barrier()


def _allreduce(x, op):
    b = _require()
    if b is None:
        return float(x)
    if b == "rccl":
        N, lib = _lib()
        v = np.array([float(x)])
        N.check(lib.gmat_comm_allreduce_f64(_state["comm"], N.ptr(v), 1, 1 if op == "max" else 0),
                "gmat_comm_allreduce_f64")
        return float(v[0])
    import torch
    import torch.distributed as tdist
    t = torch.tensor([float(x)], dtype=torch.float64)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX if op == "max" else tdist.ReduceOp.SUM)
    return float(t.item())


def allreduce_max(x):
    return _allreduce(x, "max")


def allreduce_sum(x):
    return _allreduce(x, "sum")


def snp_shard(m, rank, ws):
    """Contiguous SNP range [lo, hi) owned by `rank` for loading."""
    per = (m + ws - 1) // ws
    return min(m, rank * per), min(m, (rank + 1) * per)


def allgather_packed(local_rows, m, nb):
    """All-gather the packed .bed rows (uint8, (hi-lo) x nb) of every rank's SNP shard into
    the full (m x nb) packed panel."""
    b = _require()
    rank, ws, _ = world()
    if b is None or ws == 1:
        return np.ascontiguousarray(local_rows).reshape(-1)
    per = (m + ws - 1) // ws
    buf = np.zeros((per, nb), dtype=np.uint8)
    buf[: local_rows.shape[0]] = local_rows
    if b == "rccl":
        N, lib = _lib()
        out = np.empty((ws * per, nb), dtype=np.uint8)
        N.check(lib.gmat_comm_allgather(_state["comm"], N.ptr(buf), N.ptr(out), buf.nbytes), "gmat_comm_allgather")
        return np.ascontiguousarray(out[:m]).reshape(-1)
    import torch
    import torch.distributed as tdist
    src = torch.from_numpy(buf)
    outs = [torch.empty_like(src) for _ in range(ws)]
    tdist.all_gather(outs, src)
    return np.ascontiguousarray(torch.cat(outs, dim=0)[:m].numpy()).reshape(-1)


def broadcast_array(arr, src=0, shape=None, dtype=np.float64):
    """Broadcast a numpy array from `src` (other ranks pass arr=None with shape)."""
    b = _require()
    if b is None:
        return arr
    rank, _, _ = world()
    buf = np.ascontiguousarray(arr, dtype=dtype) if rank == src else np.empty(tuple(shape), dtype=dtype)
    if b == "rccl":
        N, lib = _lib()
        N.check(lib.gmat_comm_broadcast(_state["comm"], N.ptr(buf), buf.nbytes, int(src)), "gmat_comm_broadcast")
        return buf
    import torch
    import torch.distributed as tdist
    t = torch.from_numpy(buf.copy())
    tdist.broadcast(t, src)
    return t.numpy()


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


_HIT = np.dtype([("i", "<i8"), ("j", "<i8"), ("eff", "<f8"), ("var", "<f8"), ("chi", "<f8"), ("p", "<f8")])


def _pack_hits(local):
    if local is None or not len(local[0]):
        return np.zeros(0, dtype=_HIT)
    rec = np.empty(len(local[0]), dtype=_HIT)
    for name, col in zip(_HIT.names, local):
        rec[name] = col
    return rec


def _unpack_hits(rec):
    return tuple(np.ascontiguousarray(rec[name]) for name in _HIT.names)


def gather_hits(local, root=0):
    """Hit tuples of every rank merged on `root` (None elsewhere)."""
    b = _require()
    rank, ws, _ = world()
    if b is None or ws == 1:
        return merge_hits([local])
    if b == "rccl":
        N, lib = _lib()
        send = _pack_hits(local)
        sizes = np.zeros(ws)
        sizes[rank] = send.nbytes
        N.check(lib.gmat_comm_allreduce_f64(_state["comm"], N.ptr(sizes), ws, 0), "gmat_comm_allreduce_f64")
        total = int(sizes.sum())
        recv = np.zeros(total // _HIT.itemsize if rank == root else 0, dtype=_HIT)
        counts = np.zeros(ws, np.int64)
        need = ctypes.c_int64()
        N.check(lib.gmat_comm_gatherv(_state["comm"], N.ptr(send) if send.size else None, send.nbytes, root,
                                      N.ptr(counts), N.ptr(recv) if recv.size else None, recv.nbytes,
                                      ctypes.byref(need)), "gmat_comm_gatherv")
        if rank != root:
            return None
        parts, off = [], 0
        for r in range(ws):
            k = int(counts[r]) // _HIT.itemsize
            parts.append(_unpack_hits(recv[off:off + k]))
            off += k
        return merge_hits(parts)
    import torch.distributed as tdist
    gathered = [None] * ws if rank == root else None
    tdist.gather_object(None if local is None else tuple(np.asarray(a) for a in local), gathered, dst=root)
    return merge_hits(gathered) if rank == root else None


def shared_plan(geno, pvp, py, **kw):
    """EpiPlan on every rank with the spectral state (eigendecomposition and certificate
    searches, the plan setup's dominant cost) computed once on rank 0 and broadcast: the other
    ranks import it (gmat_epi_create_with), so the certificates are identical on every rank."""
    from .remma._scan import EpiPlan
    b = _require()
    rank, ws, _ = world()
    if b is None or ws == 1:
        return EpiPlan(geno, pvp, py, **kw)
    if rank == 0:
        plan = EpiPlan(geno, pvp, py, **kw)
        st = plan.export_state()
        allreduce_max(st.size)
        broadcast_array(st, 0, dtype=np.uint8)
        return plan
    size = int(allreduce_max(0))
    st = broadcast_array(None, 0, shape=(size,), dtype=np.uint8)
    return EpiPlan(geno, pvp, py, state=st, **kw)


def distributed_scan(scan_fn, kind, num_snp, p_cut, rows=None):
    """Run ``scan_fn(kind, my_rows, p_cut) -> (i, j, eff, var, chi, p)`` on this rank's
    share and gather the merged hits on rank 0 (other ranks get None)."""
    _require()
    rank, ws, _ = world()
    mine = rank_rows(kind, num_snp, rank, ws, rows)
    local = scan_fn(kind, mine, p_cut) if mine.size else None
    return gather_hits(local)
