"""Probe: does decoding a batch as concurrent sub-batches on separate HIP streams beat one stream?
(batch-invariant arithmetic => identical mels). Prints ms per 50-step decode for: one stream B=32; two halves
back-to-back on one stream; two halves on two streams; four quarters on four streams."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "grad-tts_amd"))
from gradtts_amd.diffusion import Diffusion  # noqa: E402
from gradtts_amd.params import synthetic_inputs, synthetic_state_dict  # noqa: E402

dev = torch.device("cuda", 0)
B, T, N = 32, 512, 50
dec = Diffusion(80, 64, 1, 64, 0.05, 20, 1000, compute_dtype=torch.bfloat16)
sd = synthetic_state_dict(seed=0, n_spks=1)
dec.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
dec = dec.to(dev)
mu, z, mask, _ = synthetic_inputs(1234, B, T)
mu, z, mask = (torch.from_numpy(a).to(dev) for a in (mu, z, mask))
streams = [torch.cuda.Stream() for _ in range(4)]


def run(parts, nstreams):
    outs = []
    cur = torch.cuda.current_stream()
    sl = [slice(i * B // parts, (i + 1) * B // parts) for i in range(parts)]
    for i, s in enumerate(sl):
        st = streams[i % nstreams] if nstreams > 1 else cur
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            outs.append(dec(z[s], mask[s], mu[s], N))
    for st in streams[:nstreams]:
        cur.wait_stream(st)
    return torch.cat(outs)


ref = run(1, 1)
for name, parts, ns in [("1x32 one stream", 1, 1), ("2x16 one stream", 2, 1), ("2x16 two streams", 2, 2),
                        ("4x8 four streams", 4, 4), ("1x32 one stream", 1, 1), ("2x16 two streams", 2, 2)]:
    run(parts, ns)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        y = run(parts, ns)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    print(f"{name:20s} {ms:8.2f} ms  {B * T / ms * 1e3:9.0f} mel-frames/s  identical={torch.equal(y, ref)}", flush=True)
