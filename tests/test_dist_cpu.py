"""The N > 1 path on CPU: gloo, world_size 2 and 3, oracle compute, product sharding/merge.

A sharded scan must return exactly the rows, order and values of the single-process scan."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import gmat_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(REPO, "tests", "golden", "tiny", "tiny")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("ws", [2, 3])
def test_sharded_scan_equals_single_process(tmp_path, ws):
    out = str(tmp_path / "res.npz")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(ws),
               OMP_NUM_THREADS="1")
    procs = []
    for r in range(ws):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "dist_worker.py"), out], env=e))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0] * ws
    res = np.load(out)
    assert float(res["mx"]) == ws - 1
    assert float(res["state_ok"]) == 1.0  # shared_plan broadcast rank 0's plan state
    snp = O.read_plink(TINY)
    ref = np.load(os.path.join(REPO, "tests", "golden", "tiny", "tiny_ref.npz"))
    y, x, col, nid = O.design_matrix(TINY + ".pheno", TINY)
    a = ref["agmat"]
    pvp, py = O.projection(y, x, col, nid, [a, a * a], ref["var"])
    for kind in ("AA", "AD", "DD"):
        exp = O.epi_scan(kind, snp, pvp, py, p_cut=0.05)
        assert exp.shape[0] > 0
        np.testing.assert_array_equal(res[kind + "_0"], exp[:, 0].astype(np.int64))
        np.testing.assert_array_equal(res[kind + "_1"], exp[:, 1].astype(np.int64))
        # values: same formula; BLAS thread counts differ between the ranks and this process
        np.testing.assert_allclose(res[kind + "_2"], exp[:, 2], rtol=1e-11)
        np.testing.assert_allclose(res[kind + "_5"], exp[:, 4], rtol=1e-9)


def test_rank_rows_partition():
    from gmat_amd.dist import rank_rows
    for kind, m in (("AA", 1407), ("AD", 1407), ("DD", 200)):
        for ws in (1, 2, 4, 8):
            parts = [rank_rows(kind, m, r, ws) for r in range(ws)]
            allr = np.sort(np.concatenate(parts))
            hi = m if kind == "AD" else m - 1
            np.testing.assert_array_equal(allr, np.arange(hi))
            if kind != "AD" and ws > 1:
                pairs = [sum(m - 1 - int(i) for i in p) for p in parts]
                assert max(pairs) / min(pairs) < 1.1  # folded split balances pair counts


def test_backend_choice_is_deterministic_and_fatal(monkeypatch):
    """Every rank derives the backend from the launch environment alone (RCCL whenever a GPU is
    visible); an RCCL setup failure raises instead of dropping that rank to gloo."""
    from gmat_amd import dist
    monkeypatch.delenv("GMAT_DIST_BACKEND", raising=False)
    assert dist.choose_backend(gpu_visible=True) == "rccl"
    assert dist.choose_backend(gpu_visible=False) == "gloo"
    assert dist.choose_backend("gloo", gpu_visible=True) == "gloo"
    monkeypatch.setenv("GMAT_DIST_BACKEND", "rccl")
    assert dist.choose_backend(gpu_visible=False) == "rccl"
    with pytest.raises(ValueError):
        dist.choose_backend("mpi")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setattr(dist, "_state", {"backend": None, "comm": None})

    def boom(rank, ws):
        raise RuntimeError("ncclCommInitRank: invalid usage")

    monkeypatch.setattr(dist, "_init_rccl", boom)
    with pytest.raises(RuntimeError, match="RCCL communicator setup failed"):
        dist.init("rccl")
    assert dist.backend() is None


def test_rendezvous_file_names_the_launch(monkeypatch):
    """The unique-id file is keyed by the launcher's pid and start time, the port, the run id and
    the restart count: a restarted or later launch never reads an earlier launch's id."""
    from gmat_amd import dist
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "r1")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    a = dist._id_file()
    assert a == dist._id_file()
    assert str(os.getppid()) in a and dist._proc_start(os.getppid()) > 0
    assert a.endswith("_%d_%d" % (os.getppid(), dist._proc_start(os.getppid())))
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    assert dist._id_file() != a
