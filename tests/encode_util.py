"""numpy restatement of the device decoder of the transport encoding (ccd_decode_enc in
ccd_pack.hip; layout in include/ccdgpu.h), shared by the CPU tests."""
import numpy as np


def up(x, a):
    return (x + a - 1) // a * a


def decode(buf):
    """numpy restatement of ccd_decode_enc: [(spectra [7][n_pix][n_obs], qa [n_pix][n_obs]), ...]"""
    buf = np.asarray(buf, dtype=np.uint8)
    nc = int(buf[:8].view(np.int64)[0])
    off = buf[8:8 * (nc + 2)].view(np.int64)
    pixo = buf[8 * (nc + 2):8 * (2 * nc + 3)].view(np.int64)
    out = []
    for c in range(nc):
        sec = buf[int(off[c]):int(off[c + 1])]
        mode, n_pix, n_obs, n_pal = (int(v) for v in sec[:16].view(np.int32))
        pal = sec[16:48].view(np.uint16)
        kept, data_off, bstride, pix_base = (int(v) for v in sec[48:80].view(np.int64))
        assert pix_base == int(pixo[c])
        plane = n_pix * n_obs
        if mode == 0:
            qa = sec[128:128 + 2 * plane].view(np.uint16).reshape(n_pix, n_obs)
            s0 = 128 + up(2 * plane, 16)
            sp = sec[s0:s0 + 14 * plane].view(np.int16).reshape(7, n_pix, n_obs)
            out.append((sp.copy(), qa.copy()))
            continue
        assert 1 <= n_pal <= 16
        koff = sec[128:128 + 4 * (n_pix + 1)].view(np.uint32).astype(np.int64)
        q0 = 128 + up(4 * (n_pix + 1), 16)
        rowb = (n_obs + 1) // 2
        q4 = sec[q0:q0 + n_pix * rowb].reshape(n_pix, rowb)
        codes = np.empty((n_pix, 2 * rowb), dtype=np.uint8)
        codes[:, 0::2] = q4 & 15
        codes[:, 1::2] = q4 >> 4
        qa = pal[codes[:, :n_obs]]
        b0 = q0 + up(n_pix * rowb, 16)
        bands = sec[b0:b0 + 14 * bstride].view(np.int16).reshape(7, bstride)
        drop = int(sec[80:84].view(np.uint32)[0])
        keep = (qa & drop) == 0
        assert int(keep.sum()) == kept == int(koff[-1])
        sp = np.full((7, n_pix, n_obs), -9999, dtype=np.int16)
        sp[:, keep] = bands[:, :kept]  # row-major boolean indexing = pixel-major kept order
        out.append((sp, qa))
    return out
