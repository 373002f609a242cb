"""Multi-rank path on CPU (gloo, world_size 2): utterances sharded across ranks, decoded independently,
gathered in order -- must equal decoding the whole batch at once (the oracle stands in for the HIP
decoder, which cannot run here; the HIP path's batch invariance is tested on the GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gradtts_amd.params import synthetic_inputs, synthetic_state_dict
from gradtts_amd.shard import gather_shards, shard, shard_bounds


def test_shard_bounds_cover_everything():
    for n in range(0, 11):
        for world in range(1, 5):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from oracle import decoder as odec
        p = odec.to_torch_params(synthetic_state_dict(seed=0))
        n, T = 3, 32                                   # ragged split: 2 + 1 utterances
        mu, z, mask, _ = synthetic_inputs(5, n, T, lengths=[32, 20, 28])
        mu, z, mask = (torch.from_numpy(a) for a in (mu, z, mask))
        with torch.no_grad():
            y = odec.reverse_diffusion(p, shard(z, rank, world), shard(mask, rank, world), shard(mu, rank, world), 2)
        full = gather_shards(y, n, world)
        if rank == 0:
            np.save(os.path.join(out_dir, "gathered.npy"), full.numpy())
    finally:
        dist.destroy_process_group()


def test_sharded_decode_equals_full_batch(tmp_path):
    from oracle import decoder as odec
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "gathered.npy")
    p = odec.to_torch_params(synthetic_state_dict(seed=0))
    mu, z, mask, _ = synthetic_inputs(5, 3, 32, lengths=[32, 20, 28])
    with torch.no_grad():
        ref = odec.reverse_diffusion(p, torch.from_numpy(z), torch.from_numpy(mask), torch.from_numpy(mu), 2).numpy()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5 * np.abs(ref).max())
