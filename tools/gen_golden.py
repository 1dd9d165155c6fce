#!/usr/bin/env python3
"""Generate the committed test fixtures under tests/golden/.

1. spectrum_kat.json: the 32 random RGB -> (c0, c1, c2) known-answer pairs plus white, copied as
   DATA from lumo's src/tracer/color/spectrum/spectrum_tests.rs:36-111 (needs /root/reference).
2. cornell_oracle.npz: small Cornell renders of the CPU oracle (both sample orders) and a
   per-path dump, so that any later change of the oracle's numbers is detected.
"""
import json, os, re, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np

REF = "/root/reference/src/tracer/color/spectrum/spectrum_tests.rs"
if os.path.exists(REF):
    txt = open(REF).read()
    body = txt[txt.index("const TEST_DATA"):]
    rows = [[float(v) for v in r.split(",")] for r in re.findall(r"\[\s*([-0-9.,\s]+?)\s*\]", body)]
    pairs = [{"rgb": rows[2 * i], "coeffs": rows[2 * i + 1]} for i in range(len(rows) // 2)]
    white = re.search(r"fn white_correct\(\).*?let rgb = \[([^\]]*)\];.*?let ans = \[([^\]]*)\];", txt, re.S)
    out = {"source": "lumo src/tracer/color/spectrum/spectrum_tests.rs:36-111",
           "tolerance": "EPSILON^(1/3) with EPSILON = 1e-10 (spectrum_tests.rs:13)",
           "random": pairs,
           "white": {"rgb": [float(v) for v in white.group(1).split(",")],
                     "coeffs": [float(v) for v in white.group(2).split(",")]}}
    assert len(pairs) == 32
    json.dump(out, open(os.path.join(ROOT, "tests/golden/spectrum_kat.json"), "w"), indent=1)
    print("wrote spectrum_kat.json")

import lumo_amd as L
import oracle_ffi as O
sc = L.Scene.cornell_box(); cam = L.Camera.cornell_box((32, 32))
tasks = L.make_tasks(32, 32, 8, 0x5EED1234)
res = {}
for mode, name in ((O.WAVEFRONT, "wavefront"), (O.LUMO_ORDER, "lumo_order")):
    bufs, r, _ = O.render_tasks(sc.desc(), cam.desc, tasks, mode, 1)
    res[name] = np.concatenate(bufs)
    res[name + "_rays"] = np.array([x.num_rays for x in r], dtype=np.uint64)
p = O.trace_paths(sc.desc(), cam.desc, tasks[1])
for k, v in p.items():
    res["paths_" + k] = v
np.savez_compressed(os.path.join(ROOT, "tests/golden/cornell_oracle.npz"), **res)
print("wrote cornell_oracle.npz")
