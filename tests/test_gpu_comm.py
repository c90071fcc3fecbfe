"""The RCCL exchange of the sharded scans (gmat_comm_*, gmat_amd/dist.py's product backend) on
the one GPU of a test box: a single-rank communicator runs every collective the sharded run
uses (all-gather of packed shards, broadcast of P, fp64 all-reduce, the hit gather) through
the same C ABI; multi-rank correctness of the sharding and merge logic is covered on CPU
(tests/test_dist_cpu.py, gloo, world sizes 2 and 3)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_single_rank_communicator():
    from gmat_amd import _native as N
    lib = N.ensure_device()
    uid = (ctypes.c_uint8 * 128)()
    N.check(lib.gmat_comm_unique_id(uid), "gmat_comm_unique_id")
    comm = ctypes.c_void_p()
    N.check(lib.gmat_comm_init(ctypes.byref(comm), 1, 0, uid), "gmat_comm_init")
    try:
        rng = np.random.default_rng(0)
        send = rng.integers(0, 255, 12345, dtype=np.uint8)
        recv = np.zeros_like(send)
        N.check(lib.gmat_comm_allgather(comm, N.ptr(send), N.ptr(recv), send.nbytes), "allgather")
        np.testing.assert_array_equal(recv, send)
        p = rng.standard_normal((300, 300))
        q = p.copy()
        N.check(lib.gmat_comm_broadcast(comm, N.ptr(q), q.nbytes, 0), "broadcast")
        np.testing.assert_array_equal(q, p)
        v = np.array([1.5, -2.0, 3.25])
        N.check(lib.gmat_comm_allreduce_f64(comm, N.ptr(v), 3, 1), "allreduce")
        np.testing.assert_array_equal(v, [1.5, -2.0, 3.25])
        counts = np.zeros(1, np.int64)
        out = np.zeros(send.size, np.uint8)
        need = ctypes.c_int64()
        N.check(lib.gmat_comm_gatherv(comm, N.ptr(send), send.nbytes, 0, N.ptr(counts), N.ptr(out), out.nbytes,
                                      ctypes.byref(need)), "gatherv")
        assert counts[0] == send.nbytes and need.value == send.nbytes
        np.testing.assert_array_equal(out, send)
        small = np.zeros(10, np.uint8)
        rc = lib.gmat_comm_gatherv(comm, N.ptr(send), send.nbytes, 0, N.ptr(counts), N.ptr(small), small.nbytes,
                                   ctypes.byref(need))
        assert rc == -5 and need.value == send.nbytes  # GMAT_E_OVERFLOW
        N.check(lib.gmat_comm_barrier(comm), "barrier")
    finally:
        lib.gmat_comm_destroy(comm)
