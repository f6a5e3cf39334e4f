"""Register / scratch report of the HIP kernels (hipcc -Rpass-analysis=kernel-resource-usage).

  python tools/kres.py [source.hip] [-D...]   -> one line per kernel: VGPRs, AGPRs, scratch, occupancy
"""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "quantized_spectrum_cartography_amd/csrc/qsc_pass.hip"
extra = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
       "-ffp-contract=off", "-fno-slp-vectorize", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = {}
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill):\s*(\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    n = r["name"]
    try:
        n = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt", n], capture_output=True,
                           text=True).stdout.strip()
    except OSError:
        pass
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    print("%-60s vgpr %4s agpr %3s scratch %4s spill %3s occ %s" % (
        n[:60], r.get("VGPRs"), r.get("AGPRs"), r.get("ScratchSize [bytes/lane]"),
        r.get("VGPRs Spill"), r.get("Occupancy [waves/SIMD]")))
