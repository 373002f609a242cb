"""The HIP decoder under ranks: 2 ranks started by torch.distributed.run, both on
cuda:0 over gloo (the 1-GPU box cannot host two RCCL ranks), each decoding its shard of 12 utterances
(6 per rank: the throughput tile plan, as on 8 GPUs at 32 per rank) and gathering the mels with
gradtts_amd.shard.gather_shards. The gathered batch must equal the single-process decode of all 12 utterances bit for
bit: per-utterance GroupNorm slots and attention tiles make the arithmetic independent of the batch an utterance is in.
(The 1 -> 8 GPU scaling curve itself is the driver's 8-GPU run; it has not been measured on hardware.)"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import gpu_available
from gpu_util import make_decoder

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def test_two_rank_hip_decode_equals_single_process(tmp_path):
    import shard_hip_worker as w
    from gradtts_amd.params import synthetic_inputs
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "gathered.npy"
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.setdefault("OMP_NUM_THREADS", "1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(HERE, "shard_hip_worker.py"),
                        str(out)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    got = torch.from_numpy(np.load(out))
    mu, z, mask, _ = synthetic_inputs(808, w.N_UTT, w.T, lengths=w.LENGTHS)
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    full = dec(*(torch.from_numpy(a).cuda() for a in (z, mask, mu)), w.STEPS).cpu()
    assert got.shape == full.shape
    assert torch.isfinite(full).all()
    assert torch.equal(got, full), float((got - full).abs().max())
