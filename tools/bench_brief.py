"""One-line summary of a bench.py JSON line (developer tool): tile, resident, roofline fracs,
the other configs' resident legs, CPU baseline."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d.get('roofline') or {}
print('tile %.0f px/s (%.2f s) parity %s | resident %.0f | frac %.4f hw %.4s valu_busy %.4s | launch %.2f ms' % (
    d['value'], d.get('tile', {}).get('seconds', 0), (d.get('tile', {}).get('parity_sample') or {}).get('int_mismatches'),
    d.get('value_resident', 0), r.get('frac', 0), r.get('hw_fp64_frac'), r.get('valu_busy'),
    r.get('kernel_ms_per_launch', 0)))
for k in sorted(x for x in d if x.startswith('resident_c')):
    v = d[k]
    print('  %s %.0f px/s, %.2f ms/launch, frac %.4f, key %s' % (k, v['value'], v['roofline']['kernel_ms_per_launch'],
                                                            v['roofline']['frac'], v['workload_key']))
if 'cpu_baseline' in d:
    print('  cpu_baseline %.1f px/s: %s' % (d['cpu_baseline']['value'], d['cpu_baseline']['sample']))
if 'tile_lossless' in d:
    print('  lossless %.0f px/s' % d['tile_lossless']['value'])
