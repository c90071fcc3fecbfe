"""Profiling driver: the configs[1] GRM and 2-GRM REML legs of bench.py alone (rocprofv3 --kernel-trace
shows one REML iteration's kernels; tools/reml_timeline.py splits the trace by iteration).
    python tools/reml_only.py [N_ID M_SNP]"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402


def main():
    n, m = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (2000, 50000)))
    g = bench.grm_bench(n, m, 1, reps=1)
    bench.reml_bench(bench.grm_bench.last_k, 1)  # first call: workspaces, streams, code objects
    r = [bench.reml_bench(bench.grm_bench.last_k, 1) for _ in range(3)]
    r.sort(key=lambda x: x["ms_per_iter"])
    print(json.dumps({"grm_kernel_ms": g["kernel_ms"], "reml": r[1]}), flush=True)


if __name__ == "__main__":
    main()
