"""Host restatement of the device chip packer (TEST INFRASTRUCTURE ONLY: imported by tests/,
never by the product path).  numpy base64 decode + pivot of the chipmunk payloads that
ccdc.chipmunk.pack_text lays out, into the detection layout of include/ccdgpu.h:
spectra [C][7][n_pix][n] int16, qa [C][n_pix][n] uint16; missing layers (offset -1) are fill
(-9999 / QA 1).  Follows merlin's pyccd format of the reference pipeline (ccdc/timeseries.py:120,
chips per ubid and date -> per-pixel arrays) with numpy's own base64 / frombuffer."""
import base64

import numpy as np


def decode(dates, text, offsets, n_pix):
    dates = np.asarray(dates)
    offsets = np.asarray(offsets)
    n_chips, n_obs = dates.shape
    enc = 4 * ((2 * n_pix + 2) // 3)
    spectra = np.empty((n_chips, 7, n_pix, n_obs), dtype=np.int16)
    qa = np.empty((n_chips, n_pix, n_obs), dtype=np.uint16)
    for c in range(n_chips):
        for o in range(n_obs):
            for l in range(8):
                off = int(offsets[c, o, l])
                if off < 0:
                    v = np.full(n_pix, 1 if l == 7 else -9999, dtype=np.uint16 if l == 7 else np.int16)
                else:
                    raw = base64.b64decode(text[off:off + enc], validate=True)
                    v = np.frombuffer(raw[:2 * n_pix], dtype='<u2' if l == 7 else '<i2')
                if l == 7:
                    qa[c, :, o] = v
                else:
                    spectra[c, l, :, o] = v
    return spectra, qa
