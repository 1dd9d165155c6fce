"""Film output (film.rs, color/space.rs TRCs, png) and tone mapping (tone_mapping.rs) in the
oracle: Clamp bounds every sample, Reinhard compresses, NoMap is the identity."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from lumo_amd.image import DCI_P3, REC_2020, encode, read_png


def test_trc_and_saturating_u8():
    c = np.array([-1.0, 0.0, 0.001, 0.0031308, 0.5, 1.0, 2.0, np.nan, np.inf])
    e = encode(c, DCI_P3)
    assert e[0] == 0 and e[1] == 0 and e[-2] == 0 and e[-1] == 255 and e[-3] == 255
    assert e[5] == int((1.055 * 1.0 - 0.055) * 255)  # 0.9999999999999999 * 255 truncates to 254 as in lumo
    assert e[2] == int(12.92 * 0.001 * 255)
    assert e[4] == int((1.055 * 0.5 ** (1 / 2.4) - 0.055) * 255)
    r = encode(np.array([0.01, 0.5]), REC_2020)
    assert r[0] == int(4.5 * 0.01 * 255)


def _film(tone_map):
    sc = L.Scene.cornell_box()
    cam = L.Camera.cornell_box((32, 32))
    tasks = L.make_tasks(32, 32, 8, 11)
    bufs, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 4, tone_map=tone_map)
    f = L.Film(32, 32)
    for t, b in zip(tasks, bufs):
        f.add_tile(t, b)
    return f


def test_tone_maps():
    base = _film(L.ToneMap.NO_MAP).rgb()
    again = _film((0, 0.0)).rgb()
    np.testing.assert_array_equal(base, again)
    reinhard = _film(L.ToneMap.REINHARD).rgb()
    assert np.nanmean(reinhard) < np.nanmean(base)
    clamped = _film(L.ToneMap.clamp(0.05)).rgb()
    assert np.nanmean(clamped) < np.nanmean(base)
    # clamped samples are bounded in the spectral domain; the filtered RGB stays finite
    assert np.isfinite(clamped).all() and np.isfinite(reinhard).all()


def test_save_png(tmp_path):
    f = _film(L.ToneMap.NO_MAP)
    p = tmp_path / "cornell.png"
    f.save(str(p))
    img = read_png(str(p))
    assert img.shape == (32, 32, 3)
    np.testing.assert_array_equal(img, f.rgb_image())
    assert img.mean() > 10
