"""Table of scripts/pmc_head.sh: per flash kernel (dispatch-averaged) MFMA busy, instruction mix,
dependency waits, LDS bank conflicts and HBM bytes.  usage: pmc_head_table.py gpurun_out/<tag>"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
# optional second argument: comma-separated kernel-name substrings to keep (default: flash kernels)
keep = sys.argv[2].split(",") if len(sys.argv) > 2 else None
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(d + "/g*/pmc_counter_collection.csv")):
    per = collections.defaultdict(float)  # (kernel, dispatch, counter) -> summed value
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if keep is not None:
            if not any(x in k for x in keep):
                continue
        elif not any(x in k for x in ("flash_", "fa3::", "fa32::")) or (
                "fwd_kernel" not in k and "cols" not in k and "rows_kernel" not in k):
            continue
        per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in per.items():
        agg[k][c].append(v)
m = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
print("| kernel | MFMA busy | VALU / MFMA | LDS / MFMA | SALU / MFMA | VMEM / MFMA | wait-on-dependency | waitcnt / barrier | issuing | LDS bank conflict / LDS active | HBM read | HBM write |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|")
for k, c in sorted(m.items()):
    g = lambda n: c.get(n, float("nan"))  # noqa: E731
    busy = g("SQ_VALU_MFMA_BUSY_CYCLES") / 1024 / (g("GRBM_GUI_ACTIVE") / 8)
    mf = g("SQ_INSTS_MFMA")
    if not mf > 0:  # no matrix work (prep / combine / sum kernels a name filter let through)
        continue
    print(f"| `{k.split('::')[-1]}` | {100 * busy:.0f} % | {g('SQ_INSTS_VALU') / mf:.2f} | {g('SQ_INSTS_LDS') / mf:.2f} | "
          f"{g('SQ_INSTS_SALU') / mf:.2f} | {g('SQ_INSTS_VMEM') / mf:.2f} | "
          f"{100 * g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.0f} % | "
          f"{100 * g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.0f} % | {100 * g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'):.0f} % | "
          f"{100 * g('SQ_LDS_BANK_CONFLICT') / max(1.0, g('SQ_LDS_IDX_ACTIVE')):.1f} % | "
          f"{g('FETCH_SIZE') / 1e6:.2f} GB | {g('WRITE_SIZE') / 1e6:.2f} GB |")
