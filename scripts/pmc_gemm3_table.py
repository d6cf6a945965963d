"""Table of scripts/pmc_gemm3.sh: per GEMM kernel and problem (dispatch-averaged) MFMA busy,
instruction mix, waits, LDS bank conflicts, L2 hit rate and HBM bytes.
usage: pmc_gemm3_table.py gpurun_out/<tag>"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(d + "/g*/pmc_counter_collection.csv")):
    per = collections.defaultdict(float)
    grid = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "gemm3_kernel" in k:
            name = "gemm3"
        elif k.startswith("Cijk"):
            name = "hipBLASLt"
        else:
            continue
        key = (name, r.get("Grid_Size", r.get("Grid_Size_X", "")))
        per[(key, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in per.items():
        agg[k][c].append(v)
m = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
print("| kernel (grid) | MFMA busy | VALU / MFMA | LDS / MFMA | SALU / MFMA | VMEM / MFMA | wait-on-dependency | waitcnt / barrier | LDS conflict | L2 hit | HBM read | HBM write |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|")
for k, c in sorted(m.items()):
    g = lambda n: c.get(n, float("nan"))  # noqa: E731
    busy = g("SQ_VALU_MFMA_BUSY_CYCLES") / 1024 / (g("GRBM_GUI_ACTIVE") / 8)
    mf = g("SQ_INSTS_MFMA")
    hit = g("TCC_HIT_sum") / max(1.0, g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    print(f"| {k[0]} ({k[1]}) | {100 * busy:.0f} % | {g('SQ_INSTS_VALU') / mf:.2f} | {g('SQ_INSTS_LDS') / mf:.2f} | "
          f"{g('SQ_INSTS_SALU') / mf:.2f} | {g('SQ_INSTS_VMEM') / mf:.2f} | "
          f"{100 * g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.0f} % | "
          f"{100 * g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.0f} % | "
          f"{100 * g('SQ_LDS_BANK_CONFLICT') / max(1.0, g('SQ_LDS_IDX_ACTIVE')):.1f} % | {100 * hit:.0f} % | "
          f"{2 * g('FETCH_SIZE') / 1e6:.2f} GB | {g('WRITE_SIZE') / 1e6:.2f} GB |")
