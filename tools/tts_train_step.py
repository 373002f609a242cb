"""One GradTTS.compute_loss + backward per iteration at the reference's training shape (params.py: batch 16,
out_size 172; ~120-190 tokens, 3-4 mel frames per token), for rocprofv3 kernel traces of the training step.
usage: python tools/tts_train_step.py [iters]"""
import os
import random
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "grad-tts_amd"), os.path.join(REPO, "tests"), REPO]
from test_tts_loss_gpu import make_gradtts  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rng = np.random.default_rng(5)
    B, Tx, out_size = 16, 190, 172
    x_lengths = rng.integers(120, Tx + 1, B)
    x_lengths[0] = Tx
    y_lengths = (x_lengths * rng.uniform(3.0, 4.0, B)).astype(np.int64)
    Ty = int(y_lengths.max())
    tokens = rng.integers(0, 149, (B, Tx)).astype(np.int64)
    y = (rng.standard_normal((B, 80, Ty)) * 1.5).astype(np.float32)
    m = make_gradtts().train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    c = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    args = (c(tokens), c(x_lengths), c(y), c(y_lengths))
    for i in range(iters + 2):
        if i == 2:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        random.seed(i)
        dur, prior, diff = m.compute_loss(*args, out_size=out_size)
        (dur + prior + diff).backward()
        opt.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    print(f"GradTTS training step (compute_loss + backward + Adam) B={B} Tx<={Tx} Ty<={Ty}: {ms:.2f} ms; losses "
          f"{float(dur):.4f} {float(prior):.4f} {float(diff):.4f}")


if __name__ == "__main__":
    main()
