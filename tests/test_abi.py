"""C-ABI checks that need no GPU: the libraries load, export every symbol the headers declare,
and the struct layouts agree between include/ccdgpu.h and the ctypes mirror."""
import ctypes
import os
import re

import pytest

import ccdgpu
from ccdgpu import abi, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, 'include', header)).read()
    return sorted(set(re.findall(r'\b(ccd(?:gpu|synth)_[a-z_]+)\s*\(', txt)))


def test_libccdgpu_exports_every_declared_symbol():
    L = ccdgpu.lib()
    names = declared('ccdgpu.h')
    assert 'ccdgpu_detect_batch' in names
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(ccdgpu.EXPORTS)


def test_libccdsynth_exports_every_declared_symbol():
    L = synth.lib()
    for n in declared('ccdsynth.h'):
        assert hasattr(L, n), n


def test_struct_sizes_and_defaults():
    assert ctypes.sizeof(abi.Segment) == 4 * 6 + 8 + 8 * (7 * 3 + 49)
    p = ccdgpu.default_params()  # host-only entry point, no device needed
    q = abi.default_params()
    for name, _ in abi.Params._fields_:
        assert getattr(p, name) == getattr(q, name), name
    assert 'gfx950' in ccdgpu.version()


def test_params_from_pyccd_dict():
    p = abi.params_from_dict({'PEEK_SIZE': 8, 'DETECTION_BANDS': [1, 3], 'CURVE_QA': {'START': 15},
                              'ADAPTIVE_PEEK': False})
    assert p.peek_size == 8 and p.detection_bands == 0b1010 and p.curve_qa_start == 15
    assert p.adaptive_peek == 0
    with pytest.raises(KeyError):
        abi.params_from_dict({'NOT_A_PARAM': 1})


def test_init_without_gpu_fails_loudly():
    """No CPU fallback: on a host with no gfx950 device the context refuses to come up."""
    if ccdgpu.device_count() > 0:
        pytest.skip('a GPU is visible')
    with pytest.raises(ccdgpu.CcdGpuError):
        ccdgpu.Context(0)
    with pytest.raises(ccdgpu.CcdGpuError):
        ccdgpu.Context(0, copy_cus=8)


def test_init_rejects_a_negative_cu_reservation():
    with pytest.raises(ccdgpu.CcdGpuError, match='copy_cus'):
        ccdgpu.Context(0, copy_cus=-1)


def test_header_constants_match_the_binding():
    txt = open(os.path.join(ROOT, 'include', 'ccdgpu.h')).read()
    assert int(re.search(r'#define CCDGPU_UPLOAD_SLOTS (\d+)', txt).group(1)) == ccdgpu.UPLOAD_SLOTS


def test_stats_struct_carries_the_pool_fields():
    names = [n for n, _ in abi.Stats._fields_]
    assert names[-4:] == ['pool_reruns', 'pool_cap', 'wave_slots', 'n_cu']
    txt = open(os.path.join(ROOT, 'include', 'ccdgpu.h')).read()
    body = txt[txt.index('typedef struct ccdgpu_stats'):txt.index('} ccdgpu_stats;')]
    assert re.findall(r'\b(\w+);', body) == names


class _FakeLib(object):
    """ccdgpu_run_slot_end_rows of a finished batch: return code ``rc``, ``rows`` rows"""

    def __init__(self, rc, rows, msg):
        self.rc, self.rows, self.msg = rc, rows, msg

    def ccdgpu_run_slot_end_rows(self, ctx, secs, nr):
        nr._obj.value = self.rows
        return self.rc

    def ccdgpu_last_error(self):
        return self.msg.encode()


@pytest.mark.parametrize('rc,msg,qa', [(abi.E_QA, 'unsupported bit-packed QA value (pixel 7)', True),
                                       (abi.E_OVERFLOW, 'run_slot_end_rows: 900 rows, the buffer holds 264', False)])
def test_run_slot_end_rows_fetches_short_rows_and_keeps_the_qa_error(monkeypatch, rc, msg, qa):
    """Context.run_slot_end_rows (ccdgpu/__init__.py) after a chain whose rows did not fit the copy:
    the rows are fetched into grown buffers whether the library says CCDGPU_EOVERFLOW or -- the
    batch also holding an unsupported QA value -- CCDGPU_EQA with the row count set; qa_error
    follows the return code (the tile runner raises on it)."""
    ctx = object.__new__(ccdgpu.Context)
    ctx.qa_error = False
    ctx._ctx = None
    bufs = ccdgpu.RowsBuffers(pinned=False, rows_per_pixel=0.5)
    ctx._rows_req = ([0], [0], bufs, 100, 400, 13, 264)
    ctx._pending_slot = 0
    ctx._slot_keep = {0: object()}
    fetched = []
    ctx.fetch_batch_rows_into = lambda cx, cy, b, w: fetched.append(b) or ('rows',)
    monkeypatch.setattr(ccdgpu, 'lib', lambda: _FakeLib(rc, 900, msg))
    out = ctx.run_slot_end_rows()
    assert out == ('rows',) and fetched == [bufs]
    assert ctx.qa_error is qa
    assert bufs.rows_per_pixel >= 1.25 * 900 / 400
