"""MFMA-pipe utilisation per kernel from a rocprofv3 --pmc pass of SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY (scripts/gpu_full.sh).

mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs): GRBM_GUI_ACTIVE is summed over
the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES counts cycles (32 per v_mfma_f32_32x32x16_bf16, MI355X_MICROARCH.md).
wait_any / wave_cycles: the fraction of wave lifetime parked on s_waitcnt / barriers.

usage: python scripts/pmc_mfma.py gpurun_out/pmc_mfma_<tag>/run_counter_collection.csv [top]
"""
import collections
import csv
import re
import sys

top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name).split("(")[0]
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
rows = []
for name, c in acc.items():
    gui = c.get("GRBM_GUI_ACTIVE", 0.0)
    if gui <= 0 or c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) <= 0:
        continue
    util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8.0 * 256 * 4)
    wait = c.get("SQ_WAIT_ANY", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0)
    rows.append((c["SQ_VALU_MFMA_BUSY_CYCLES"], name, util, wait))
print(f"{'kernel':78s} {'mfma_util':>9s} {'wait_any/wave_cycles':>21s}")
for _, name, util, wait in sorted(rows, reverse=True)[:top]:
    print(f"{name[:78]:78s} {util:9.3f} {wait:21.2f}")
