"""Summarise tools/gpu_pack_pmc.sh output: per-launch counters of the largest unpack launches
(8 chips) and the derived traffic / VALU figures.  Usage: pack_pmc_summary.py gpurun_out/TAG"""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
per = collections.defaultdict(list)
for f in sorted(glob.glob(f'{tag}_p*/run_counter_collection.csv')):
    agg, grid = collections.defaultdict(float), {}
    for r in csv.DictReader(open(f)):
        if 'unpack' not in r['Kernel_Name']:
            continue
        agg[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
        grid[r['Dispatch_Id']] = int(r['Grid_Size'])
    big = max(grid.values())
    for (d, c), v in agg.items():
        if grid[d] == big:
            per[c].append(v)
m = {c: sum(v) / len(v) for c, v in per.items()}
for c in sorted(m):
    print(f'{c:22s} {m[c]:.4g}')
ms = [float(r['AverageNs']) for r in csv.DictReader(open(f'{tag}_stats/run_kernel_stats.csv')) if 'unpack' in r['Name']]
print('stats average ns (all launches):', ms)
if 'FETCH_SIZE' in m and 'WRITE_SIZE' in m:
    print(f"HBM read {2 * m['FETCH_SIZE'] * 1024 / 1e9:.3f} GB (FETCH_SIZE x 2), write {m['WRITE_SIZE'] * 1024 / 1e9:.3f} GB")
if 'SQ_WAVES' in m:
    w = m['SQ_WAVES']
    print(f"per wave: VALU {m['SQ_INSTS_VALU'] / w:.0f}  LDS {m['SQ_INSTS_LDS'] / w:.0f}  SALU {m.get('SQ_INSTS_SALU', 0) / w:.0f}")
if 'GRBM_GUI_ACTIVE' in m and 'SQ_ACTIVE_INST_VALU' in m:
    print(f"VALU busy {m['SQ_ACTIVE_INST_VALU'] * 4 / (4 * 256 * m['GRBM_GUI_ACTIVE'] / 8):.2f}")
