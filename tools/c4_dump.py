"""Config 4 (B = 4096, N = 64, seed 46) solved on the GPU, everything saved for analysis on the
CPU: python tools/c4_dump.py OUT.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    N, B = 64, 4096
    model = default_model()
    h = _lib.Handle(model, N=N, max_batch=B, qp_mode=_lib.QP_BOX)
    xcur, goals, XU = make_batch(h, model, B, N, seed=46)
    out, st = h.solve(xcur, goals, XU)
    it, conv, mu = h.box_stats(B)
    np.savez_compressed(sys.argv[1], xcur=xcur, goals=goals, XU=XU, out=out, qp_iters=st["qp_iters"],
                        alphas=st["alphas"], n_alphas=st["n_alphas"], ipm_iters=it, ipm_conv=conv, ipm_mu=mu)
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()
