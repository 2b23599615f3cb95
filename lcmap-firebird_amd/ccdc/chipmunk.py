"""ccdc.chipmunk -- chipmunk wire format -> the device chip packer.

The reference builds its per-pixel records with ``merlin.create`` (ccdc/timeseries.py:120),
which fetches every ARD layer's chips from chipmunk (base64 100x100 int16/uint16 payloads, one
per ubid and acquisition date: fixtures test/data/chip_response.json, registry_response.json),
pivots them per pixel on the Spark executors and then reshuffles the pixels
(``repartition``, timeseries.py:125).  Here a chip's payloads stay text until they reach HBM:
``group`` sorts the chips of one location into layers and dates, ``pack_text`` concatenates
the payloads with their byte offsets, and ``ccdgpu.Context.stage_chipmunk`` decodes and pivots
them on the device (lcmap-firebird_amd/csrc/ccd_pack.hip) straight into the detection layout.
Nothing is decoded on the host.

``ARD_UBIDS`` restates the layer -> ubid map of lcmap-merlin's ``chipmunk-ard`` profile
(external dependency, not in /root/reference; [ext], unverified against its pinned source):
surface reflectance bands and band-10 brightness temperature of Landsat 4, 5, 7 and 8, and the
pixel QA.  ``check_registry`` pins it against the reference's own registry fixture: every ubid
exists there with the band tags this mapping implies.  Date handling follows merlin's pyccd
format: the dates of all layers must agree (``symmetric``) and come out descending, the order
merlin delivers (timeseries.py:115 example).
"""
from datetime import date, datetime

import numpy as np

LAYERS = ('blues', 'greens', 'reds', 'nirs', 'swir1s', 'swir2s', 'thermals', 'qas')

ARD_UBIDS = {
    'blues':    ('LC08_SRB2', 'LE07_SRB1', 'LT05_SRB1', 'LT04_SRB1'),
    'greens':   ('LC08_SRB3', 'LE07_SRB2', 'LT05_SRB2', 'LT04_SRB2'),
    'reds':     ('LC08_SRB4', 'LE07_SRB3', 'LT05_SRB3', 'LT04_SRB3'),
    'nirs':     ('LC08_SRB5', 'LE07_SRB4', 'LT05_SRB4', 'LT04_SRB4'),
    'swir1s':   ('LC08_SRB6', 'LE07_SRB5', 'LT05_SRB5', 'LT04_SRB5'),
    'swir2s':   ('LC08_SRB7', 'LE07_SRB7', 'LT05_SRB7', 'LT04_SRB7'),
    'thermals': ('LC08_BTB10', 'LE07_BTB6', 'LT05_BTB6', 'LT04_BTB6'),
    'qas':      ('LC08_PIXELQA', 'LE07_PIXELQA', 'LT05_PIXELQA', 'LT04_PIXELQA'),
}

# registry tags each layer's ubids must carry, and their data type
_LAYER_TAGS = {'blues': ('sr', 'blue'), 'greens': ('sr', 'green'), 'reds': ('sr', 'red'),
               'nirs': ('sr', 'nir'), 'swir1s': ('sr', 'swir1'), 'swir2s': ('sr', 'swir2'),
               'thermals': ('bt',), 'qas': ('pixelqa',)}
_LAYER_TYPE = {name: ('UINT16' if name == 'qas' else 'INT16') for name in LAYERS}

CHIP_PIXELS = 10000  # 100 x 100 30 m pixels (grid_response.json: 3000 m chips)


def _layer_of():
    return {u.lower(): name for name, ubids in ARD_UBIDS.items() for u in ubids}


def check_registry(registry):
    """Check ARD_UBIDS against a chipmunk registry (list of {ubid, tags, data_type, ...}):
    raises ValueError naming the first ubid that is absent, mistyped or mis-tagged."""
    by = {e['ubid'].lower(): e for e in registry}
    for name, ubids in ARD_UBIDS.items():
        for u in ubids:
            e = by.get(u.lower())
            if e is None:
                raise ValueError('ubid %s (%s) is not in the registry' % (u, name))
            tags = set(t.lower() for t in e.get('tags') or ())
            if not set(_LAYER_TAGS[name]) <= tags:
                raise ValueError('ubid %s (%s) lacks tags %s' % (u, name, _LAYER_TAGS[name]))
            if e.get('data_type') != _LAYER_TYPE[name]:
                raise ValueError('ubid %s (%s) is %s, not %s' % (u, name, e.get('data_type'), _LAYER_TYPE[name]))
    return True


def ordinal(acquired):
    """chipmunk 'acquired' timestamp (ISO 8601, e.g. 2002-12-21T00:00:00Z) -> proleptic ordinal."""
    s = str(acquired)
    try:
        return datetime.strptime(s[:10], '%Y-%m-%d').date().toordinal()
    except ValueError:
        return date.fromisoformat(s[:10]).toordinal()


def group(chips):
    """chipmunk chip dicts {x, y, acquired, ubid, data, ...} (any order, any locations) ->
    {(x, y): {layer: {ordinal: base64 payload}}}.  Chips of ubids outside ARD_UBIDS are
    ignored; two payloads for the same location, layer and date are an error."""
    layer_of = _layer_of()
    out = {}
    for c in chips:
        name = layer_of.get(str(c['ubid']).lower())
        if name is None:
            continue
        key = (int(c['x']), int(c['y']))
        d = ordinal(c['acquired'])
        layers = out.setdefault(key, {n: {} for n in LAYERS})
        if d in layers[name]:
            raise ValueError('two %s chips for %s on %s' % (name, key, date.fromordinal(d)))
        layers[name][d] = c['data']
    return out


def dates_of(layers, symmetric=True):
    """Descending acquisition ordinals of one location's layers.  symmetric: every layer must
    hold the same dates (merlin's symmetric date check); otherwise the union is returned and
    absent layers stage as fill."""
    sets = [set(layers[n]) for n in LAYERS]
    union = set().union(*sets)
    if symmetric and any(s != union for s in sets):
        missing = {n: sorted(union - s)[:3] for n, s in zip(LAYERS, sets) if s != union}
        raise ValueError('asymmetric dates across layers: %r' % (missing,))
    return np.array(sorted(union, reverse=True), dtype=np.int64)


def pack_text(locations, symmetric=True):
    """[layers, ...] of chips sharing one date vector (values of ``group``) ->
    (dates [C][n] int64 descending, text bytes, offsets [C][n][8] int64) for
    ccdgpu.Context.stage_chipmunk.  Offsets are byte offsets of each payload in text, -1 for a
    missing layer (only when symmetric=False)."""
    dates = [dates_of(l, symmetric) for l in locations]
    for d in dates[1:]:
        if not np.array_equal(d, dates[0]):
            raise ValueError('chips of one batch must share their acquisition dates')
    n_obs = dates[0].shape[0]
    offsets = np.full((len(locations), n_obs, len(LAYERS)), -1, dtype=np.int64)
    parts, pos = [], 0
    for c, layers in enumerate(locations):
        for o, d in enumerate(dates[c]):
            for l, name in enumerate(LAYERS):
                payload = layers[name].get(int(d))
                if payload is None:
                    continue
                b = payload.encode('ascii') if isinstance(payload, str) else bytes(payload)
                offsets[c, o, l] = pos
                parts.append(b)
                pos += len(b)
    return np.stack(dates), b''.join(parts), offsets


def payload_pixels(payload):
    """Number of 16-bit values a base64 payload decodes to."""
    b = payload.encode('ascii') if isinstance(payload, str) else bytes(payload)
    pad = len(b) - len(b.rstrip(b'='))
    return (len(b) // 4 * 3 - pad) // 2


def encode(values):
    """One layer of one date as its chipmunk payload (base64 of little-endian 16-bit values);
    for building synthetic chipmunk responses."""
    import base64
    v = np.ascontiguousarray(values)
    dt = '<u2' if v.dtype.kind == 'u' else '<i2'
    return base64.b64encode(v.astype(dt).tobytes()).decode('ascii')


def chip_response(x, y, dates, spectra, qa):
    """Synthetic chipmunk response for one location: dates [n] ordinals, spectra [7][n_pix][n]
    int16, qa [n_pix][n] uint16 -> list of chip dicts (one per layer and date, Landsat 7 ubids
    before 2013-04-11 and Landsat 8 ubids after, as chipmunk would serve them)."""
    out = []
    l8 = date(2013, 4, 11).toordinal()
    for o, d in enumerate(np.asarray(dates, dtype=np.int64)):
        sensor = 0 if d >= l8 else 1
        acq = date.fromordinal(int(d)).isoformat() + 'T00:00:00Z'
        for l, name in enumerate(LAYERS):
            vals = qa[:, o] if name == 'qas' else spectra[l, :, o]
            out.append({'x': int(x), 'y': int(y), 'acquired': acq, 'ubid': ARD_UBIDS[name][sensor].lower(),
                        'data': encode(vals)})
    return out
