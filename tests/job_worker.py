"""Worker for tests/test_job_cpu.py: one rank of a gloo (CPU) job exercising the multi-rank drop-in
API helpers of gmat_amd/dist.py (no GPU: the device calls are replaced by host stand-ins).

Writes <out>.rank<r>.json with what this rank saw; the test compares the ranks."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gmat_amd import dist  # noqa: E402


def main():
    out = sys.argv[1]
    work = sys.argv[2]
    rank, ws = dist.job()
    rec = {"rank": rank, "ws": ws}

    # root_call: rank 0 alone runs the function (and writes its file); every rank gets the result and
    # rank 0's np.random state (rank 0 draws, the others do not)
    np.random.seed(100 + rank)
    calls = []

    @dist.on_root
    def write_and_draw(path):
        calls.append(1)
        with open(path, "w") as f:
            f.write("written by rank %d\n" % rank)
        return {"draw": np.random.randint(1 << 30, size=3).tolist()}

    res = write_and_draw(os.path.join(work, "root_file"))
    rec["root_result"] = res
    rec["root_calls"] = len(calls)
    rec["after_root_draw"] = int(np.random.randint(1 << 30))
    with open(os.path.join(work, "root_file")) as f:
        rec["root_file"] = f.read()

    # nested sections run locally on rank 0 (no collective inside a rank-0 section)
    @dist.on_root
    def outer():
        return inner() + 1

    @dist.on_root
    def inner():
        return 41

    rec["nested"] = outer()

    # an exception on rank 0 reaches every rank as the same exception type
    @dist.on_root
    def bad():
        raise ValueError("snp_lst_0 is out of range!")

    try:
        bad()
        rec["raised"] = None
    except ValueError as exc:
        rec["raised"] = str(exc)

    # sharded genotype read: every rank's shard all-gathered is the whole .bed body
    from gmat_amd.plink import read_bed_body
    tiny = os.path.join(REPO, "tests", "golden", "tiny", "tiny")
    body, n, m = read_bed_body(tiny)
    lo, hi = dist.snp_shard(m, rank, ws)
    rows, n2, m2 = dist.read_bed_rows(tiny, lo, hi)
    full = dist.allgather_packed(rows, m, (n + 3) // 4)
    rec["bed_gather_ok"] = bool(np.array_equal(full, body) and (n2, m2) == (n, m))

    # row shards: the whole triangle -> the folded split; a subset -> contiguous runs of equal pairs
    m_ = 1000
    full_rows = np.arange(m_ - 1)
    sub = np.arange(100, 700, 3)
    rec["shard_full"] = dist.shard_rows("AA", m_, full_rows, rank, ws).tolist()
    rec["shard_sub"] = dist.shard_rows("AA", m_, sub, rank, ws).tolist()
    rec["shard_ad"] = dist.shard_rows("AD", m_, sub, rank, ws).tolist()

    # gather_records: list order kept across the ranks
    b = dist.split_weighted(np.ones(11), ws)
    mine = np.arange(11)[b[rank]:b[rank + 1]]
    r = np.zeros(mine.size, dtype=[("x", "<f8"), ("k", "<i8")])
    r["x"] = mine * 0.5
    r["k"] = mine
    g = dist.gather_records(r)
    rec["gathered"] = None if g is None else g["k"].tolist()

    # the effect screen's part files: each rank screens its contiguous run, rank 0 joins them
    from gmat_amd.remma import _eff

    def fake_screen(sym, args, temp_file):
        rws, path = args
        with open(path, "w") as f:
            f.write("snp_0 snp_1 eff\n")
            for i in rws.tolist():
                f.write("%d %d %s\n" % (i, i + 1, sym))

    _eff._screen = fake_screen
    rows_eff = np.array([5, 3, 9, 1, 7, 2, 8], dtype=np.longlong)
    tf = os.path.join(work, "eff.temp")
    _eff._screen_parts("AA", "S", lambda rr, t: (rr, t), 20, rows_eff, tf)
    if rank == 0:
        with open(tf) as f:
            rec["eff_temp"] = f.read()
        rec["leftover_parts"] = sorted(x for x in os.listdir(work) if ".part" in x)
    dist.barrier()
    with open("%s.rank%d.json" % (out, rank), "w") as f:
        json.dump(rec, f)


if __name__ == "__main__":
    main()
