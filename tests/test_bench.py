"""bench.py's roofline bookkeeping on CPU: the committed PMC records (profiles/pmc_*.json) carry
the fields the bench line reads and are found by their workload keys, and the hardware FP64
fraction the bench reports is reproducible from a record and the committed kernel-stats average."""
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_pmc_records_are_found_by_their_workload_keys():
    paths = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'pmc_*.json')))
    assert any(p.endswith('pmc_detect.json') for p in paths)
    keys = set()
    for p in paths:
        rec = json.load(open(p))
        for k in ('workload', 'hbm_bytes_per_launch', 'hbm_read_bytes', 'hbm_write_bytes', 'counters'):
            assert k in rec, (p, k)
        assert rec['hbm_bytes_per_launch'] == rec['hbm_read_bytes'] + rec['hbm_write_bytes']
        assert rec['workload'] not in keys, 'two records for one workload key'
        keys.add(rec['workload'])
        found, got = bench.pmc_record(rec['workload'])
        assert found == os.path.relpath(p, ROOT) and got == rec
    assert bench.pmc_record('no such workload') == (None, {})


def test_hardware_fp64_fraction_reproduces_from_the_committed_profiles():
    rec = json.load(open(os.path.join(ROOT, 'profiles', 'pmc_detect.json')))
    c = rec['counters']
    rows = list(csv.DictReader(open(os.path.join(ROOT, 'profiles', 'r06', 'kernel_stats.csv'))))
    det = [r for r in rows if 'ccd_detect' in r['Name']]
    assert len(det) == 1
    ms = float(det[0]['AverageNs']) * 1e-6
    hw = bench.hardware_fp64(c, ms, 256)
    lane = 64 * (c['SQ_INSTS_VALU_ADD_F64'] + c['SQ_INSTS_VALU_MUL_F64'] + 2 * c['SQ_INSTS_VALU_FMA_F64']
                 + c['SQ_INSTS_VALU_TRANS_F64'])
    assert hw['lane_flops'] == lane
    assert abs(hw['frac'] - lane / (ms * 1e-3) / (bench.FP64_PEAK_TFLOPS * 1e12)) < 1e-12
    assert 0.0 < hw['frac'] < 1.0 and 0.0 < hw['valu_issue_model'] <= hw['valu_busy'] < 1.0
    assert bench.hardware_fp64({}, ms, 256) == {}
