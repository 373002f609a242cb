"""Worker of test_shard_hip_gpu.py (not collected): one rank of a 2-rank torch.distributed.run job, both ranks on
cuda:0 over gloo (RCCL refuses two ranks on one device) -- the GRADTTS_BENCH_SHARED_DEVICE arrangement of bench.py.
Each rank decodes its utterance shard with the HIP decoder (bf16, throughput plan: 6 utterances per rank) and the
mels are gathered with gradtts_amd.shard.gather_shards; rank 0 saves the gathered batch to argv[1]."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "grad-tts_amd"))

from gpu_util import make_decoder  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402
from gradtts_amd.shard import gather_shards, shard  # noqa: E402

N_UTT, T, STEPS = 12, 256, 3
LENGTHS = [256, 200, 256, 131, 256, 97, 256, 180, 211, 256, 140, 256]


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    try:
        torch.cuda.set_device(0)
        mu, z, mask, _ = synthetic_inputs(808, N_UTT, T, lengths=LENGTHS)
        mu, z, mask = (torch.from_numpy(a).cuda() for a in (mu, z, mask))
        dec, _ = make_decoder(1, 0, torch.bfloat16)
        y = dec(shard(z, rank, world), shard(mask, rank, world), shard(mu, rank, world), STEPS)
        full = gather_shards(y, N_UTT, world)
        if rank == 0:
            np.save(sys.argv[1], full.cpu().numpy())
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
