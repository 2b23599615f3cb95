"""Summarise rocprofv3 --pmc passes (gpurun_out/<tag>_p*/run_counter_collection.csv) for the
detection kernel: per-dispatch counter values, HBM bytes per launch (FETCH_SIZE doubled per the
MI355X guide's gfx950 correction + WRITE_SIZE), derived rates.  Developer tool (runs here)."""
import csv, glob, json, os, sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "pmc"
root = "gpurun_out"
kern = 'ccd_detect'
vals = defaultdict(list)
dur = []
for f in sorted(glob.glob(os.path.join(root, tag + '_p*', 'run_counter_collection.csv'))):
    per = defaultdict(float)
    for row in csv.DictReader(open(f)):
        if kern not in row['Kernel_Name']:
            continue
        per[(row['Dispatch_Id'], row['Counter_Name'])] += float(row['Counter_Value'])
        if row['Counter_Name'] == 'GRBM_GUI_ACTIVE':
            dur.append((int(row['End_Timestamp']) - int(row['Start_Timestamp'])) * 1e-9)
    for (d, c), v in per.items():
        vals[c].append(v)
out = {c: sum(v) / len(v) for c, v in vals.items()}
if 'FETCH_SIZE' in out:  # KB units; gfx950 reports half the bytes of wide reads
    out['hbm_read_bytes'] = out['FETCH_SIZE'] * 1024 * 2
if 'WRITE_SIZE' in out:
    out['hbm_write_bytes'] = out['WRITE_SIZE'] * 1024
if 'hbm_read_bytes' in out and 'hbm_write_bytes' in out:
    out['hbm_bytes_per_launch'] = out['hbm_read_bytes'] + out['hbm_write_bytes']
if dur:
    out['kernel_s'] = sum(dur) / len(dur)
    if 'GRBM_GUI_ACTIVE' in out:
        out['clock_ghz'] = out['GRBM_GUI_ACTIVE'] / 8 / out['kernel_s'] / 1e9
for a, b in (('SQ_WAIT_ANY', 'SQ_WAVE_CYCLES'), ('SQ_ACTIVE_INST_ANY', 'SQ_WAVE_CYCLES'),
             ('SQ_WAIT_INST_ANY', 'SQ_WAVE_CYCLES'), ('TCC_HIT_sum', 'TCC_MISS_sum')):
    if a in out and b in out and out[b]:
        out[a + '/' + b] = out[a] / out[b]
print(json.dumps(out, indent=1))

# --write <workload> [--out pmc_<name>.json]: record the per-launch HBM traffic and counters for
# bench.py's roofline (bench.py reads every profiles/pmc_*.json and matches 'workload')
if '--write' in sys.argv:
    wl = sys.argv[sys.argv.index('--write') + 1]
    rec = {'workload': wl, 'kernel': kern, 'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tag %s' % tag,
           'hbm_bytes_per_launch': out.get('hbm_bytes_per_launch'),
           'hbm_read_bytes': out.get('hbm_read_bytes'), 'hbm_write_bytes': out.get('hbm_write_bytes'),
           'correction': 'FETCH_SIZE x 2 (gfx950 reports half the bytes of wide reads, MI355X_MICROARCH.md HBM section); WRITE_SIZE as read',
           'counters': {k: v for k, v in out.items() if k.isupper() or k.startswith('SQ_') or k.startswith('TC')}}
    os.makedirs(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles'), exist_ok=True)
    name = sys.argv[sys.argv.index('--out') + 1] if '--out' in sys.argv else 'pmc_detect.json'
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles', name)
    json.dump(rec, open(path, 'w'), indent=1)
    print('wrote', path)
