"""Per-kernel rocprof averages of the configs[2] steps of a `rocprofv3 --kernel-trace -- python3 bench.py` run,
next to the bench line's own HIP-event figures, so that the two can be compared (the stats CSV averages
over every leg of the run: configs[4], the split parts, the parity rows).
   python tools/bench_trace_summary.py run_kernel_trace.csv bench.json"""
import csv
import json
import sys

from step_timeline import short

KERNELS = ("prefilter_pass_kernel", "lrc_screen_kernel", "pair_side_kernel", "pair_mxr_kernel", "refine8_kernel",
           "refine8_side_kernel")


def main():
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                  for r in csv.DictReader(open(sys.argv[1])))
    b = json.load(open(sys.argv[2]))
    warm, steps = b["warmup"], b["steps"]
    # the configs[2] scans come first in the run: warmup + timed steps, one refine8_kernel each
    fins = [k for k, e in enumerate(rows) if e[2].startswith("refine8_fin_kernel")]
    n_scan = warm + steps
    end = rows[fins[n_scan - 1]][1]
    t0 = rows[fins[warm - 1]][1] if warm > 0 else 0
    print("rocprofv3 --kernel-trace -- python3 bench.py (warmup %d, steps %d); bench line: ms_per_step %.3f, "
          "roofline kernel %s avg_launch_ms %.4f (HIP events)"
          % (warm, steps, b["ms_per_step"], b["roofline"]["kernel"], b["roofline"]["avg_launch_ms"]))
    for name in KERNELS:
        allk = [e for e in rows if e[2].startswith(name) and e[1] <= end]
        timed = [e for e in allk if e[0] >= t0]
        if not timed:
            continue
        ev = b["roofline"]["kernels"].get(name, {}).get("avg_launch_ms")
        print("%-22s the %d timed steps: %3d launches, average %8.1f us (rocprof)%s" % (
            name, steps, len(timed), sum(e[1] - e[0] for e in timed) / len(timed) / 1e3,
            "; HIP events %.1f us" % (ev * 1e3) if ev else ""))


if __name__ == "__main__":
    main()
