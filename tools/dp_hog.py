"""Is one process's train-step gradient repeatable while ANOTHER process keeps the GPU busy? (GPU dev tool)

The DP tests run two ranks on one GPU. tools/dp_diag.py found each rank's local gradient sometimes differing
from one process's, while the exchange itself was always exact. This probe takes the second rank's role away:
one process computes the same local gradient REPS times (fresh model each time, bitwise compare with the
first) while a background process runs unrelated GPU work (bf16 matmuls) — or nothing (`--alone`).

    python tools/dp_hog.py CONFIG DTYPE B REPS [--alone]
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402


def hog(seconds):
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    t0 = time.time()
    while time.time() - t0 < seconds:
        for _ in range(20):
            a = (a @ a).clamp_(-1, 1)
        torch.cuda.synchronize()


def main():
    if sys.argv[1] == "--hog":
        hog(float(sys.argv[2]))
        return
    config, dtype, B, reps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    alone = "--alone" in sys.argv
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import det_probe as D
    bg = None if alone else subprocess.Popen([sys.executable, __file__, "--hog", "120"])
    try:
        time.sleep(0 if alone else 5)
        g0, offs = D.local_grad(config, dtype, B)
        for i in range(1, reps):
            g, _ = D.local_grad(config, dtype, B)
            D.report(f"rep {i}{' (alone)' if alone else ' (beside a busy process)'}", g, g0, offs)
    finally:
        if bg is not None:
            bg.kill()
            bg.wait()


if __name__ == "__main__":
    main()
