"""Load tests/golden/*.npz (written by tests/golden/make_golden.py) as abi.Unpacked-like objects."""
import glob
import json
import os

import numpy as np

from ccdgpu import abi

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, '*.npz')))


def load(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + '.npz'))  # allow_pickle=False (default)
    d, s, q = z['dates'], z['spectra'], z['qa']
    params = json.loads(str(z['params']))
    u = abi.Unpacked()
    u.n_pix, u.n_obs = q.shape
    u.seg_offsets = z['seg_offsets']
    u.segments = z['segments']
    u.mask = np.unpackbits(z['mask'], axis=1, bitorder='little')[:, :u.n_obs].astype(bool)
    u.procedure = z['procedure']
    u.probs = z['probs']
    # the restatement's date sort (numpy's quicksort tie order unless ARGSORT 'stable')
    order = z['sort_index'].astype(np.int64) if 'sort_index' in z.files else np.argsort(d, kind='stable')
    u.sorted_dates = d[order]
    u.sort_index = order.astype(np.int32)
    u.error_pixel = -1
    u.seconds_kernel = u.seconds_total = 0.0
    return (d, s, q), params, u
