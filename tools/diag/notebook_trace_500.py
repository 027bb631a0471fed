"""Diagnostic: the GPU closed loop (i7m_mpc_run, B = 1) over the notebook's full 500 steps vs the
goal distances pin_mpc_indy7.ipynb printed (reference OSQP at eps 1e-3)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from indy7_mpc_amd import _lib  # noqa: E402
from indy7_mpc_amd.model import default_model  # noqa: E402

tr = json.load(open(os.path.join(ROOT, "tests", "golden", "notebook_kats.json")))["mpc_trace"]
m = default_model()
h = _lib.Handle(m, N=32, max_batch=1)
ends = h.eepos(np.array(tr["endpoint_q"]))
d, q, xc, xu = h.mpc_run(np.array([tr["xstart"]]), ends, 500)
ref = np.array(tr["goal_distances"])
dd = np.abs(d[:, 0] - ref)
for a, b in ((0, 8), (8, 50), (50, 100), (100, 200), (200, 300), (300, 400), (400, 500)):
    print(f"steps {a:3d}-{b:3d}: max |d - ref| {dd[a:b].max():.3e}  max rel {(dd[a:b] / ref[a:b]).max():.3e}")
print("final", d[-1, 0], ref[-1], "min gpu", np.nanmin(d[:, 0]), "min ref", ref.min(), "argmax ref", int(ref.argmax()),
      "argmax gpu", int(np.nanargmax(d[:, 0])))
