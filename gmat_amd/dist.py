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
import contextlib
import ctypes
import functools
import os
import pickle
import sys
import tempfile
import time

import numpy as np

_state = {"backend": None, "comm": None, "root_depth": 0, "failed": False}


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
            global _prev_hook
            if sys.excepthook is not _note_failure:
                _prev_hook, sys.excepthook = sys.excepthook, _note_failure
    _state["backend"] = backend
    return backend


def _note_failure(exc_type, exc, tb):
    """sys.excepthook: a rank dying on an exception skips the exit barrier (its peers wait in another
    collective, or are gone: the barrier would hold the failing rank for gloo's 30-minute timeout)."""
    _state["failed"] = True
    _prev_hook(exc_type, exc, tb)


_prev_hook = sys.__excepthook__


def _destroy_gloo():
    import torch.distributed as tdist
    if not tdist.is_initialized():
        return
    try:
        if not _state.get("failed"):
            # clean exit: wait for the peers (a rank leaving first tears its sockets down under a peer's
            # last collective), bounded so that a peer that died without an exception cannot hold us
            import datetime
            try:
                tdist.monitored_barrier(timeout=datetime.timedelta(seconds=60))
            except Exception:
                pass
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
    rec = gather_records(_pack_hits(local), root)
    return merge_hits([_unpack_hits(rec)]) if rank == root else None


def shared_plan(geno, pvp, py, **kw):
    """EpiPlan on every rank with the spectral state (eigendecomposition and certificate
    searches, the plan setup's dominant cost) computed once on rank 0 and broadcast: the other
    ranks import it (gmat_epi_create_with), so the certificates are identical on every rank."""
    from .remma._scan import EpiPlan
    rank, ws = job()
    if ws == 1:
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


# ---------------------------------------------------------------- the drop-in API as one multi-rank job
#
# A user script run as N ranks (torchrun, ``python -m gmat_amd.launch --gpus N script.py`` or
# GMAT_NUM_GPUS=N) executes every line on every rank.  The reference's functions then behave as one job:
# * the exhaustive scans, the pair lists and the effect screens shard their work over the ranks and
#   rank 0 alone writes the output files (remma/_scan.py, remma/_eff.py);
# * everything single-GPU (GRM, REML, projections, single-SNP tests, annotation, random pairs) runs on
#   rank 0 only and its result is broadcast (root_call): the files exist before any rank returns, and
#   the other ranks get the same return value;
# * the global np.random state is rank 0's on every rank after each such call, as if every rank had
#   made it (imputation of missing calls and the unseeded random pairs draw from it).


def job():
    """(rank, world_size) of the drop-in API: the process group is set up on first use when
    WORLD_SIZE > 1.  Inside a rank-0-only section (root_call) this is (0, 1): a nested call runs as a
    single process."""
    rank, ws, _ = world()
    if ws <= 1 or _state["root_depth"] > 0:
        return 0, 1
    init()
    return rank, ws


@contextlib.contextmanager
def local():
    """Inside: the drop-in API runs as a single process on this rank (no collectives), e.g. bench.py's
    rank-0-only legs."""
    _state["root_depth"] += 1
    try:
        yield
    finally:
        _state["root_depth"] -= 1


def broadcast_bytes(data, src=0):
    """A byte string from `src` to every rank (others pass None)."""
    rank, ws = job()
    if ws == 1:
        return data
    size = np.array([len(data) if rank == src else 0], dtype=np.int64)
    size = broadcast_array(size, src, shape=(1,), dtype=np.int64)
    n = int(size[0])
    if n == 0:
        return b""
    buf = np.frombuffer(data, dtype=np.uint8) if rank == src else None
    return broadcast_array(buf, src, shape=(n,), dtype=np.uint8).tobytes()


def broadcast_object(obj, src=0):
    """A Python object of this process's own making (never a file's content) from `src`."""
    rank, ws = job()
    if ws == 1:
        return obj
    data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL) if rank == src else None
    return pickle.loads(broadcast_bytes(data, src))


def sync_rng(src=0):
    """The global np.random state of `src` on every rank."""
    rank, ws = job()
    if ws > 1:
        np.random.set_state(broadcast_object(np.random.get_state() if rank == src else None, src))


def root_call(fn, *args, **kw):
    """fn(*args, **kw) on rank 0 only; every rank returns its result (or raises its exception) and
    leaves with rank 0's np.random state.  A single process just calls fn."""
    rank, ws = job()
    if ws == 1:
        return fn(*args, **kw)
    payload = None
    if rank == 0:
        _state["root_depth"] += 1
        try:
            payload = ("ok", fn(*args, **kw))
        except BaseException as exc:  # noqa: B902 -- re-raised below on every rank
            try:
                pickle.dumps(exc)
                payload = ("err", exc)
            except Exception:
                payload = ("err", RuntimeError("rank 0: %s: %s" % (type(exc).__name__, exc)))
        finally:
            _state["root_depth"] -= 1
        payload = payload + (np.random.get_state(),)
    status, value, state = broadcast_object(payload)
    np.random.set_state(state)
    if status == "err":
        raise value
    return value


def on_root(fn):
    """Decorator: the function runs as root_call(fn, ...)."""
    @functools.wraps(fn)
    def wrapper(*args, **kw):
        return root_call(fn, *args, **kw)
    wrapper.__wrapped_root__ = fn
    return wrapper


def split_weighted(weights, ws):
    """Contiguous bounds b[0] = 0 <= ... <= b[ws] = len(weights) splitting `weights` (pairs per row)
    into ws runs of about equal sum (list order kept: concatenating the runs gives the list back)."""
    w = np.asarray(weights, dtype=np.float64)
    if w.size == 0:
        return np.zeros(ws + 1, dtype=np.int64)
    cum = np.concatenate([[0.0], np.cumsum(w)])
    targets = cum[-1] * np.arange(ws + 1) / ws
    b = np.searchsorted(cum, targets, side="left").astype(np.int64)
    b[0], b[-1] = 0, w.size
    return np.maximum.accumulate(b)


def row_pairs(kind, num_snp, rows):
    """Pairs a scan of first SNP i tests: m - 1 - i (AA / DD, j > i), m (AD, every j)."""
    rows = np.asarray(rows, dtype=np.int64)
    return np.full(rows.size, num_snp, np.int64) if kind == "AD" else num_snp - 1 - rows


def shard_rows(kind, num_snp, rows, rank, ws):
    """This rank's share of the sorted unique first-SNP rows of a scan: the reference's folded split
    (rank_rows) when the rows are the whole triangle, else a contiguous run of about 1/ws of the pairs."""
    rows = np.asarray(rows, dtype=np.int64)
    if ws == 1:
        return rows
    hi = num_snp if kind == "AD" else num_snp - 1
    if rows.size == hi and (hi == 0 or (rows[0] == 0 and rows[-1] == hi - 1)):
        return rank_rows(kind, num_snp, rank, ws)
    b = split_weighted(row_pairs(kind, num_snp, rows), ws)
    return rows[b[rank]:b[rank + 1]]


def read_bed_rows(bed_file, lo, hi):
    """Packed .bed rows [lo, hi) (uint8, (hi - lo) x nb) read from their offset, the magic and the
    whole file's size checked as plink.read_bed_body does; returns (rows, n_id, n_snp)."""
    from .plink import BED_MAGIC, count_lines
    n = count_lines(bed_file + ".fam")
    m = count_lines(bed_file + ".bim")
    nb = (n + 3) // 4
    with open(bed_file + ".bed", "rb") as f:
        magic = f.read(3)
        if magic != BED_MAGIC:
            raise ValueError("%s.bed is not a SNP-major PLINK .bed (magic %r)" % (bed_file, magic))
        size = os.fstat(f.fileno()).st_size - 3
        if size < nb * m:
            raise ValueError("%s.bed has %d data bytes; %d SNPs x %d individuals need %d"
                             % (bed_file, size, m, n, nb * m))
        f.seek(3 + lo * nb)
        rows = np.frombuffer(f.read((hi - lo) * nb), dtype=np.uint8).reshape(hi - lo, nb)
    return rows, n, m


def load_geno(bed_file):
    """The device genotype panel of a .bed fileset on every rank: each rank reads its SNP shard and
    the packed shards are all-gathered (RCCL over xGMI); missing calls are imputed on the whole panel
    with the (synchronised) global np.random state, so every rank holds the same panel, the one a
    single process would impute (process_plink.py:12-25)."""
    from .plink import Geno
    rank, ws = job()
    if ws == 1:
        return Geno(bed_file)
    from .plink import count_lines
    m = count_lines(bed_file + ".bim")
    lo, hi = snp_shard(m, rank, ws)
    local, n, m = read_bed_rows(bed_file, lo, hi)
    body = allgather_packed(local, m, (n + 3) // 4)
    sync_rng()
    return Geno(body=body, n_id=n, n_snp=m)


def gather_records(rec, root=0):
    """A structured numpy array from every rank, concatenated in rank order on `root` (None
    elsewhere)."""
    b = _require()
    rank, ws, _ = world()
    if b is None or ws == 1:
        return rec
    if b == "rccl":
        N, lib = _lib()
        send = np.ascontiguousarray(rec)
        recv_n = None
        sizes = np.zeros(ws)
        sizes[rank] = send.nbytes
        N.check(lib.gmat_comm_allreduce_f64(_state["comm"], N.ptr(sizes), ws, 0), "gmat_comm_allreduce_f64")
        recv_n = int(sizes.sum()) // rec.dtype.itemsize
        recv = np.zeros(recv_n if rank == root else 0, dtype=rec.dtype)
        counts = np.zeros(ws, np.int64)
        need = ctypes.c_int64()
        N.check(lib.gmat_comm_gatherv(_state["comm"], N.ptr(send) if send.size else None, send.nbytes, root,
                                      N.ptr(counts), N.ptr(recv) if recv.size else None, recv.nbytes,
                                      ctypes.byref(need)), "gmat_comm_gatherv")
        return recv if rank == root else None
    import torch.distributed as tdist
    gathered = [None] * ws if rank == root else None
    tdist.gather_object(np.ascontiguousarray(rec), gathered, dst=root)
    return np.concatenate(gathered) if rank == root else None
