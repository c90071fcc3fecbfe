"""The drop-in API as one multi-rank job, on CPU (gloo): the launch paths (GMAT_NUM_GPUS,
``python -m gmat_amd.launch``), the rank-0 sections (root_call), the sharded reads and the
order-keeping merges of gmat_amd/dist.py, and a failing rank ending the job at once.
The GPU side (the README workflow's scans as 2 ranks, byte-identical files) is
tests/test_gpu_multirank.py."""
import json
import os
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest

from gmat_amd import dist, launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "MASTER_ADDR", "GMAT_DIST_BACKEND",
                        "GMAT_NUM_GPUS")}
    env["OMP_NUM_THREADS"] = "1"
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    env.update(**kw)
    return env


RANK_SCRIPT = """
import os, sys
import gmat_amd
print("rank %s of %s args %s" % (os.environ["RANK"], os.environ["WORLD_SIZE"], sys.argv[1:]), flush=True)
"""


def test_gmat_num_gpus_runs_the_script_as_ranks(tmp_path):
    """GMAT_NUM_GPUS=2 python script.py a b: the import of gmat_amd starts two ranks of the same
    command line, and the parent exits with their status without running the rest of the script."""
    script = tmp_path / "s.py"
    script.write_text(RANK_SCRIPT)
    out = subprocess.run([sys.executable, str(script), "a", "b"], env=_env(GMAT_NUM_GPUS="2"), cwd=str(tmp_path),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = sorted(l for l in out.stdout.splitlines() if l.startswith("rank"))
    assert lines == ["rank 0 of 2 args ['a', 'b']", "rank 1 of 2 args ['a', 'b']"]


def test_gmat_num_gpus_refuses_stdin(tmp_path):
    out = subprocess.run([sys.executable, "-"], input="import gmat_amd\nprint('ran')\n", env=_env(GMAT_NUM_GPUS="2"),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 2 and "needs a script" in out.stderr and "ran" not in out.stdout


def test_launch_module_cli(tmp_path):
    script = tmp_path / "s.py"
    script.write_text(RANK_SCRIPT)
    out = subprocess.run([sys.executable, "-m", "gmat_amd.launch", "--gpus", "3", str(script), "--flag", "x"],
                         env=_env(), cwd=REPO, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = sorted(l for l in out.stdout.splitlines() if l.startswith("rank"))
    assert lines == ["rank %d of 3 args ['--flag', 'x']" % r for r in range(3)]


def test_failing_rank_after_init_ends_the_job_fast(tmp_path):
    """A rank raising after dist.init() leaves at once (no exit barrier on the error path) while its
    peer waits in a collective: the launcher returns the failure within seconds, not gloo's 30 min."""
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent("""
        import os
        from gmat_amd import dist
        dist.init("gloo")
        if os.environ["RANK"] == "1":
            raise RuntimeError("rank 1 fails")
        dist.allreduce_sum(1.0)  # waits for rank 1 in another collective than an exit barrier
    """))
    t0 = time.time()
    rc = launch.spawn([sys.executable, str(script)], 2, environ=_env())
    assert rc != 0
    assert time.time() - t0 < 60


def test_clean_exit_is_fast(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent("""
        from gmat_amd import dist
        dist.init("gloo")
        dist.barrier()
    """))
    t0 = time.time()
    assert launch.spawn([sys.executable, str(script)], 2, environ=_env()) == 0
    assert time.time() - t0 < 60


def test_check_devices_probe_failure():
    assert launch.check_devices(2, None, False) and "could not be probed" in launch.check_devices(2, None, False)
    assert launch.check_devices(2, None, True) is None


def test_split_weighted_and_shards():
    w = np.arange(100, 0, -1)
    for ws in (1, 2, 3, 8):
        b = dist.split_weighted(w, ws)
        assert b[0] == 0 and b[-1] == w.size and np.all(np.diff(b) >= 0)
        sums = [w[b[k]:b[k + 1]].sum() for k in range(ws)]
        assert max(sums) - min(sums) <= 2 * w.max()
    assert dist.split_weighted([], 4).tolist() == [0] * 5
    assert dist.split_weighted(np.ones(3), 5)[-1] == 3


@pytest.mark.parametrize("ws", [2, 3])
def test_job_helpers_over_gloo(tmp_path, ws):
    work = tmp_path / "work"
    work.mkdir()
    out = str(tmp_path / "res")
    rc = launch.spawn([sys.executable, os.path.join(REPO, "tests", "job_worker.py"), out, str(work)], ws,
                      environ=_env())
    assert rc == 0
    recs = [json.load(open("%s.rank%d.json" % (out, r))) for r in range(ws)]
    r0 = recs[0]
    for r, rec in enumerate(recs):
        assert rec["rank"] == r and rec["ws"] == ws
        assert rec["root_result"] == r0["root_result"]  # rank 0's result everywhere
        assert rec["root_calls"] == (1 if r == 0 else 0)
        assert rec["after_root_draw"] == r0["after_root_draw"]  # rank 0's np.random state everywhere
        assert rec["root_file"] == "written by rank 0\n"
        assert rec["nested"] == 42
        assert rec["raised"] == "snp_lst_0 is out of range!"
        assert rec["bed_gather_ok"]
    np.random.seed(100)
    exp_draw = np.random.randint(1 << 30, size=3).tolist()
    assert r0["root_result"] == {"draw": exp_draw}
    full = np.concatenate([rec["shard_full"] for rec in recs])
    np.testing.assert_array_equal(np.sort(full), np.arange(999))
    for key, kind in (("shard_sub", "AA"), ("shard_ad", "AD")):
        cat = np.concatenate([rec[key] for rec in recs])
        np.testing.assert_array_equal(cat, np.arange(100, 700, 3))  # contiguous runs in order
        pairs = [float(np.sum(dist.row_pairs(kind, 1000, rec[key]))) for rec in recs]
        assert max(pairs) - min(pairs) <= 1000
    assert r0["gathered"] == list(range(11)) and all(rec["gathered"] is None for rec in recs[1:])
    exp = "snp_0 snp_1 eff\n" + "".join("%d %d S\n" % (i, i + 1) for i in (5, 3, 9, 1, 7, 2, 8))
    assert r0["eff_temp"] == exp and r0["leftover_parts"] == []
