"""bench.py --gpus N without an external launcher (gmat_amd/launch.py).

CPU: the launch decision, two ranks reaching dist.init() over gloo through bench.py itself,
failure propagation, the device-count check.  GPU: --gpus N beyond the visible GPUs is refused; the
real sharded scan through the same launcher (two ranks on the box's one GPU, --allow-shared-gpu,
exchanges over gloo) at the bench's full cohort gives the one-rank step's hits byte for byte."""
import json
import os
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest

from gmat_amd import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _clean_env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "MASTER_ADDR", "GMAT_DIST_BACKEND")}
    env["OMP_NUM_THREADS"] = "1"
    env.update(**kw)
    return env


def test_resolve():
    assert launch.resolve(1, {}) == "single"
    assert launch.resolve(4, {}) == "spawn"
    assert launch.resolve(4, {"WORLD_SIZE": "4"}) == "rank"
    assert launch.resolve(1, {"WORLD_SIZE": "1"}) == "single"
    with pytest.raises(launch.LaunchError):
        launch.resolve(8, {"WORLD_SIZE": "1"})  # driver asked for 8, the launcher made 1: never silent
    with pytest.raises(launch.LaunchError):
        launch.resolve(2, {"WORLD_SIZE": "4"})
    with pytest.raises(launch.LaunchError):
        launch.resolve(0, {})


def test_rank_env():
    env = launch.rank_env({"X": "1"}, 3, 8, 29511)
    assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"], env["MASTER_PORT"]) == ("3", "3", "8", "29511")
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["X"] == "1"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_gpus2_reaches_dist_init_on_two_ranks():
    """python bench.py --gpus 2 (no WORLD_SIZE): two ranks join one gloo group on this CPU box."""
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], env=_clean_env(), cwd=REPO,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 2 and rec["rank_sum"] == 1.0 and rec["backend"] == "gloo"
    assert rec["launcher"] == "gmat_amd.launch"


def test_bench_refuses_mismatched_world_size():
    env = _clean_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--dry-run"], env=env, cwd=REPO,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


def test_failing_rank_stops_the_job(tmp_path):
    """Rank 1 fails at once, rank 0 would run for a minute: the launcher returns rank 1's code and
    terminates rank 0."""
    script = tmp_path / "worker.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(7)
        time.sleep(60)
    """))
    t0 = time.time()
    rc = launch.spawn([sys.executable, str(script)], 2, environ=_clean_env())
    assert rc == 7
    assert time.time() - t0 < 30


def test_check_devices():
    assert launch.check_devices(8, 8, False) is None
    assert launch.check_devices(2, 8, False) is None
    assert launch.check_devices(8, 0, False) is None  # no GPU at all: the CPU (gloo) harness
    assert launch.check_devices(8, 1, True) is None   # --allow-shared-gpu
    msg = launch.check_devices(8, 1, False)
    assert msg and "only 1 GPU" in msg


@pytest.mark.gpu
def test_bench_refuses_more_ranks_than_gpus():
    """bench.py --gpus 8 on a box with fewer GPUs exits with status 2 before starting any rank (it
    would otherwise report 8 GPUs with ranks sharing devices)."""
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--steps", "1", "--warmup", "0"], env=_clean_env(),
                         cwd=REPO, capture_output=True, text=True, timeout=240)
    n = launch.visible_devices(_clean_env())
    assert n >= 1
    if n < 8:
        assert out.returncode == 2, (out.returncode, out.stderr[-2000:])
        assert "only %d GPU" % n in out.stderr


@pytest.mark.gpu
def test_bench_gpus2_sharded_full_cohort_identical(tmp_path):
    """configs[3]'s sharded path at the bench's full size (2,000 x 50,000, p_cut 1e-5) through
    bench.py's own launcher: two ranks (on this box's one GPU, --allow-shared-gpu: the exchanges go over
    gloo) each scan part k of the reference's folded split (remma_epiAA.py:109-161) and rank 0 merges
    the hits.  The merged (i, j, eff, var, chi, p) tuples are byte-identical to the one-rank step's,
    and both equal the exhaustive (unscreened) full-triangle hit set (parity.full_triangle)."""
    common = ["--steps", "1", "--warmup", "1", "--no-cpu", "--no-grm", "--no-eff", "--no-e2e", "--no-cov",
              "--no-split", "--no-cfg5"]
    res, hits = {}, {}
    for g in (1, 2):
        path = str(tmp_path / ("hits%d.npz" % g))
        extra = ["--allow-shared-gpu"] if g > 1 else []
        out = subprocess.run([sys.executable, BENCH, "--gpus", str(g), "--hits-out", path] + extra + common,
                             env=_clean_env(OMP_NUM_THREADS="16"), cwd=REPO, capture_output=True, text=True,
                             timeout=420)
        assert out.returncode == 0, out.stderr[-3000:]
        res[g] = json.loads(out.stdout.strip().splitlines()[-1])
        hits[g] = np.load(path)
    assert res[2]["n_gpus"] == 2 and res[1]["n_gpus"] == 1
    assert res[2]["devices_used"] == min(2, launch.visible_devices(_clean_env()))
    assert res[2]["backend"] == "gloo" and res[1]["backend"] == "single"
    for g in (1, 2):
        ft = res[g]["parity"]["full_triangle"]
        assert ft["checked"], ft
        assert ft["identical"] and ft["values_byte_identical"] and ft["symmetric_difference"] == 0, ft
    assert hits[1]["i"].size == res[1]["scan"]["hits_per_step"] > 10000
    for key in ("i", "j", "eff", "var", "chi", "p"):
        a, b = hits[1][key], hits[2][key]
        assert a.dtype == b.dtype and a.shape == b.shape, key
        np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64), err_msg=key)
