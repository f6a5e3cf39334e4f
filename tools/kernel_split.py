"""Split a rocprofv3 kernel-stats CSV (--kernel-trace --stats) into the build's HIP passes, the
one-off set-up kernels and everything else (the torch / MIOpen decoder of the DIP path), per
iteration:

  python tools/kernel_split.py <..._kernel_stats.csv> <iterations> [out.json]

Used for config 5's DIP iteration (bench.py --config c5dip / tools/dip_iter.py): how much of an
iteration is the fused HIP passes and how much the decoder's forward / backward and optimizer.
"""
import csv
import json
import re
import sys

# the per-iteration HIP kernels of the DIP solver (qmc.GeneratorSolver)
PASSES = ("cpass_tile_kernel", "cpass_kernel", "cfinish_kernel", "spass_kernel", "flush_kernel",
          "perm_gather_kernel", "perm_scatter_kernel", "scfused_kernel")
# one-off kernels of the observation packing / problem set-up
SETUP = ("sched_kernel", "obs_", "pack_codes", "layout", "fill_", "order_", "count_",
         "nsq_part_kernel", "state_init_kernel", "quantize", "bin_codes", "map_", "reconstruct",
         "split_kernel", "selftest", "device_check")


def short(name):
    m = re.search(r"(\w+_kernel\w*|\w+)(?=<|\()", name)
    return m.group(1) if m else name[:60]


def split(path, iters):
    out = {"passes": {}, "setup": {}, "other": {}}
    for row in csv.DictReader(open(path)):
        name, calls, tot = row["Name"], int(row["Calls"]), float(row["TotalDurationNs"])
        s = short(name)
        if any(p in s for p in PASSES):
            cat = "passes"
        elif any(p in s for p in SETUP):
            cat = "setup"
        else:
            cat = "other"
        d = out[cat].setdefault(s, {"calls": 0, "total_us": 0.0})
        d["calls"] += calls
        d["total_us"] += tot * 1e-3
    res = {"iterations": iters}
    for cat in ("passes", "other"):
        tot = sum(v["total_us"] for v in out[cat].values())
        res[cat + "_us_per_iter"] = tot / iters
        res[cat + "_top"] = sorted(((k, round(v["total_us"] / iters, 2), v["calls"])
                                   for k, v in out[cat].items()), key=lambda x: -x[1])[:12]
    res["setup_us_total"] = sum(v["total_us"] for v in out["setup"].values())
    res["passes_share"] = res["passes_us_per_iter"] / max(
        res["passes_us_per_iter"] + res["other_us_per_iter"], 1e-30)
    return res


if __name__ == "__main__":
    r = split(sys.argv[1], int(sys.argv[2]))
    s = json.dumps(r, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
