"""Average in-sequence kernel durations from a rocprofv3 --kernel-trace --stats summary of the
bench command (the timed iteration sequence), for bench.py's roofline (measured_in_sequence):

  python tools/inseq.py <kernel_stats.csv> profiles/rNN/inseq.json [head_sha]
"""
import csv
import json
import re
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    ks = {}
    for row in csv.DictReader(open(src)):
        m = re.search(r"(\w+_kernel)(?=<|\()", row["Name"])
        if not m:
            continue
        name = m.group(1)
        calls, tot = int(row["Calls"]), float(row["TotalDurationNs"])
        d = ks.setdefault(name, {"calls": 0, "total_ns": 0.0})
        d["calls"] += calls
        d["total_ns"] += tot
    res = {"kernels": {k: {"avg_us": v["total_ns"] / v["calls"] * 1e-3, "calls": v["calls"]}
                       for k, v in ks.items() if k in ("scfused_kernel", "cfinish_kernel",
                                                       "spass_kernel", "cpass_tile_kernel")},
           "source": src, "head": sys.argv[3] if len(sys.argv) > 3 else None,
           "note": "averages over every launch of the traced bench process: the timed replays "
                   "dominate the scfused / cfinish counts"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["kernels"]))


if __name__ == "__main__":
    main()
