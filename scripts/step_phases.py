"""Median phase spans of the emulated rank step (forward kernels + combine, backward kernel pair,
tail after the backward) per rocprofv3 kernel trace; steps split at the [q|v] projection.

    python scripts/step_phases.py gpurun_out/X/*/prof_kernel_trace.csv
"""
import csv, sys, statistics
def load(p):
    rows=[]
    with open(p) as f:
        for d in csv.DictReader(f):
            rows.append((int(d['Start_Timestamp']),int(d['End_Timestamp']),d['Kernel_Name'].split('(')[0]))
    rows.sort(); return rows
for p in sys.argv[1:]:
    rows=load(p)
    idx=[i for i,r in enumerate(rows) if 'gemm_proj_kernel<1, 64, 128, false' in r[2]]
    res={'step':[],'fwd':[],'bwd':[],'tail':[]}
    for a,b in zip(idx[3:-1],idx[4:]):
        st=rows[a:b]; t0=rows[a][0]; t1=rows[b][0]
        fw=[r for r in st if 'flash_fwd_kernel' in r[2] or 'flash_fwd_combine' in r[2]]
        bw=[r for r in st if 'flash_bwd_cols2' in r[2] or 'flash_bwd_rows_kernel' in r[2]]
        res['step'].append((t1-t0)/1e3)
        res['fwd'].append((max(r[1] for r in fw)-min(r[0] for r in fw))/1e3)
        res['bwd'].append((max(r[1] for r in bw)-min(r[0] for r in bw))/1e3)
        res['tail'].append((t1-max(r[1] for r in bw))/1e3)
    print(p.split('/')[-2], {k: round(statistics.median(v),1) for k,v in res.items()}, len(res['step']))
