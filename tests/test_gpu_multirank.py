"""The drop-in API as one multi-rank job on the GPU (north star "shards SNP-pair
tiles across the GPUs" through the functions the examples call).

tests/multirank_workflow.py -- a reference-style script through ``import gmat`` -- runs unchanged
as one process and as 2 and 3 ranks of one job (``python -m gmat_amd.launch --gpus N
--allow-shared-gpu``: the box has one GPU, so the ranks share it and exchange over gloo; with one GPU
per rank the same code exchanges over RCCL).  The sharded scans, pair list and effect screen must
write exactly the files a single process writes, byte for byte, each file once (no per-rank files
left behind), and those files must match the reference's own outputs (tests/golden/mouse)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from test_gpu_parity import _cmp_hits

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOUSE = os.path.join(REPO, "tests", "golden", "mouse")
SCRIPT = os.path.join(REPO, "tests", "multirank_workflow.py")


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "MASTER_ADDR", "GMAT_NUM_GPUS")}
    env["OMP_NUM_THREADS"] = "8"
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    return env


def _run(out_dir, n):
    os.makedirs(out_dir)
    cmd = [sys.executable, SCRIPT, out_dir, MOUSE]
    if n > 1:
        cmd = [sys.executable, "-m", "gmat_amd.launch", "--gpus", str(n), "--allow-shared-gpu"] + cmd[1:]
    out = subprocess.run(cmd, env=_env(), cwd=REPO, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    assert out.stdout.count("workflow done") == n
    return {f: open(os.path.join(out_dir, f), "rb").read() for f in sorted(os.listdir(out_dir))}


@pytest.fixture(scope="module")
def runs(tmp_path_factory):
    base = tmp_path_factory.mktemp("multirank")
    return {n: _run(str(base / ("ranks%d" % n)), n) for n in (1, 2, 3)}


@pytest.mark.parametrize("n", [2, 3])
def test_ranks_write_the_single_process_files(runs, n):
    one, many = runs[1], runs[n]
    assert sorted(many) == sorted(one)  # each file once: no part files, no per-rank copies
    for name in ("epiAA_1e-5", "epiAA_1e-3", "epiAD_1e-5", "epiDD_1e-5", "epiAA_par3_1e-4.1", "epiAA_par3_1e-4.2",
                 "epiAA_par3_1e-4.3", "epiAA_pair5000", "epiAA_rows", "epiAA_eff_rows200", "epiAA_approx",
                 "epiAA_1e-3.anno", "plink.agrm0", "plink.dgrm_as0", "var_a_axa.txt"):
        assert name in one, name
        assert many[name] == one[name], name  # byte-identical


def test_single_process_files_match_the_reference(runs, tmp_path):
    d = tmp_path / "one"
    d.mkdir()
    for name, data in runs[1].items():
        (d / name).write_bytes(data)
    for name in ("epiAA_1e-5", "epiAA_1e-3", "epiAD_1e-5", "epiDD_1e-5", "epiAA_par3_1e-4.1", "epiAA_par3_1e-4.2",
                 "epiAA_par3_1e-4.3"):
        _cmp_hits(str(d / name), os.path.join(MOUSE, name))
    _cmp_hits(str(d / "epiAA_pair5000"), os.path.join(MOUSE, "epiAA_pair5000"))
    # annotation of this run's hits: the rows and .bim columns of the reference's file, floats within 1e-5
    got = [l.split() for l in (d / "epiAA_1e-3.anno").read_text().splitlines()]
    exp = [l.split() for l in open(os.path.join(MOUSE, "epiAA_1e-3.anno")).read().splitlines()]
    assert got[0] == exp[0] and len(got) == len(exp) > 1
    for a, b in zip(got[1:], exp[1:]):
        assert a[:14] == b[:14]
        np.testing.assert_allclose(np.array(a[14:], float), np.array(b[14:], float), rtol=1e-5)
    # the caller's row order and duplicates replayed (rows 700, 3, 3, 1200, 5)
    firsts = np.loadtxt(str(d / "epiAA_rows"), skiprows=1, ndmin=2)[:, 0].astype(int).tolist()
    asked = [700, 3, 3, 1200, 5]
    per_row = {r: firsts.count(r) // asked.count(r) for r in set(asked)}
    assert firsts == [r for r in asked for _ in range(per_row[r])] and len(firsts) > 0
