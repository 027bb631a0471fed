"""Per-kernel launch durations under the diagnostic I7M_ABLATE builds (results invalid, timing
only) at small and large batch, one SQP iteration per solve so that every launch
works on every problem whatever the ablation does to the results: python tools/ablate_ab.py [ablate ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.small_batch_ab import run  # noqa: E402

if __name__ == "__main__":
    for a in (sys.argv[1:] or ["0", "1", "11"]):
        for B in (1, 64, 4096):
            r = run(B, 32, {"I7M_ABLATE": a}, steps=100 if B == 1 else 20, max_sqp_iters=1)
            print("ablate", a, "B=%d" % B, r["kernels_us"], flush=True)
