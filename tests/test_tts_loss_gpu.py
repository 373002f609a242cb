"""GradTTS.compute_loss (model/tts.py:110-194) on the MI355X: the text encoder's training pass
(gt_text_encoder_forward_train / gt_text_encoder_backward), the alignment, the crop, mu_y, the auxiliary losses and
the decoder's training step, all through the library.

Tolerances (written here):
* against the REAL reference (tests/golden/tts_loss_*.npz, eval mode, fp64 reference gradients): each loss rel 1e-5
  of the reference's fp32 value; every parameter gradient's digest (norm and random projection,
  oracle.decoder.grad_digest) within 5e-5 of the reference's fp64 gradient relative to that tensor's norm (+ 1e-3 of
  the largest norm) -- fp32 through six transformer layers and the U-Net (measured <= 6.6e-6);
* train mode (dropout on, the library's masks restated by oracle.text_encoder.dropout_keep): mu_x / logw 1e-5 x
  max|ref|, encoder parameter gradients under random upstream gradients as above (5e-5; elementwise 5e-5 x max|ref|
  of each tensor), against torch.autograd through oracle/text_encoder.py in fp64;
* two calls bit-identical (fixed-order reductions).
"""
import random

import numpy as np
import pytest
import torch

from conftest import gpu_available, load_golden
from gpu_util import rel_err, report
from gradtts_amd.params import synthetic_state_dict, synthetic_text_encoder_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def make_gradtts(seed_enc=5, seed_dec=0):
    from gradtts_amd.tts import GradTTS
    m = GradTTS(149, 1, 64, 192, 768, 256, 2, 6, 3, 0.1, 4, 80, 64, 0.05, 20.0, 1000)
    sd = {f"encoder.{k}": torch.from_numpy(v) for k, v in synthetic_text_encoder_state_dict(seed_enc).items()}
    sd.update({f"decoder.estimator.{k}": torch.from_numpy(v) for k, v in synthetic_state_dict(seed=seed_dec).items()})
    m.load_state_dict(sd, strict=True)
    return m.cuda()


class fixed_draws:
    """torch.rand -> t, torch.randn -> z (the decoder's two draws, diffusion.py:284 / :249) inside the block."""

    def __init__(self, t, z):
        self.t, self.z = t, z

    def __enter__(self):
        self.orig = (torch.rand, torch.randn)

        def rand(*shape, dtype=None, device=None, requires_grad=False, **kw):
            return self.t.to(dtype=dtype or torch.float32, device=device).clone()

        def randn(*shape, dtype=None, device=None, requires_grad=False, **kw):
            shape = tuple(shape[0]) if len(shape) == 1 and not isinstance(shape[0], int) else shape
            assert tuple(shape) == tuple(self.z.shape), shape
            return self.z.to(dtype=dtype or torch.float32, device=device).clone()

        torch.rand, torch.randn = rand, randn

    def __exit__(self, *exc):
        torch.rand, torch.randn = self.orig
        return False


def run_fixture(m, g):
    out_size = int(g["out_size"])
    random.seed(int(g["py_seed"]))
    with fixed_draws(torch.from_numpy(g["t"]), torch.from_numpy(g["z"])):
        dur, prior, diff = m.compute_loss(torch.from_numpy(g["tokens"]).cuda(), torch.from_numpy(g["x_lengths"]).cuda(),
                                          torch.from_numpy(g["y"]).cuda(), torch.from_numpy(g["y_lengths"]).cuda(),
                                          out_size=out_size if out_size > 0 else None)
    return dur, prior, diff


@pytest.mark.parametrize("name", ["tts_loss_B2.npz", "tts_loss_B3_nocut.npz", "tts_loss_B2_short.npz"])
def test_compute_loss_matches_reference_fixture(name):
    from oracle import decoder as odec
    g = load_golden(name)
    m = make_gradtts(int(g["seed_enc"]), int(g["seed_dec"])).eval()
    dur, prior, diff = run_fixture(m, g)
    (dur + prior + diff).backward()
    ref = g["losses_f32"]
    for i, (nm, v) in enumerate((("dur_loss", dur), ("prior_loss", prior), ("diff_loss", diff))):
        report(f"compute_loss {nm} vs reference {name}", abs(float(v) - ref[i]) / abs(ref[i]), 1e-5)
    names = [str(n) for n in g["param_names"]]
    params = dict(m.named_parameters())
    grads = {k: params[k].grad.detach().cpu().numpy().astype(np.float64) for k in names}
    gsq, gproj = odec.grad_digest(grads, names)
    rn = np.sqrt(g["gsq_f64"])
    floor = 1e-3 * rn.max()
    err = np.maximum(np.abs(np.sqrt(gsq) - rn), np.abs(gproj - g["gproj_f64"])) / (rn + floor)
    enc = np.array([n.startswith("encoder.") for n in names])
    report(f"compute_loss encoder grad digests vs reference {name} (worst "
           f"{names[int(np.where(enc, err, -1).argmax())]})", float(err[enc].max()), 5e-5)
    report(f"compute_loss decoder grad digests vs reference {name} (worst "
           f"{names[int(np.where(~enc, err, -1).argmax())]})", float(err[~enc].max()), 5e-5)
    for k in list(g):
        if k.startswith("full__"):
            report(f"compute_loss grad {k[6:]} vs reference", rel_err(grads[k[6:]], g[k]), 5e-5)


def test_compute_loss_deterministic():
    g = load_golden("tts_loss_B2.npz")
    m = make_gradtts(int(g["seed_enc"]), int(g["seed_dec"])).train()
    res = []
    for _ in range(2):
        m.zero_grad()
        torch.manual_seed(11)
        dur, prior, diff = run_fixture(m, g)
        (dur + prior + diff).backward()
        res.append([float(dur), float(prior), float(diff)] +
                   [p.grad.detach().clone() for p in m.parameters() if p.grad is not None])
    assert res[0][:3] == res[1][:3]
    assert all(torch.equal(a, b) for a, b in zip(res[0][3:], res[1][3:]))


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_text_encoder_training_pass_matches_oracle(p_drop):
    """Train mode with dropout p (prenet 0.5): forward values and the gradients of every encoder parameter under
    random upstream gradients of mu_x and logw, against autograd through the oracle with the same masks (fp64)."""
    from oracle import text_encoder as ote
    from oracle.decoder import grad_digest
    m = make_gradtts()
    enc = m.encoder.train() if p_drop > 0 else m.encoder.eval()
    enc.p_dropout = p_drop
    rng = np.random.default_rng(7)
    lengths = [29, 17, 23]
    B, Tx = len(lengths), 29
    tokens = rng.integers(0, 149, size=(B, Tx)).astype(np.int64)
    gmu = rng.standard_normal((B, 80, Tx))
    glw = rng.standard_normal((B, 1, Tx))
    torch.manual_seed(3)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p_drop > 0 else 0
    torch.manual_seed(3)
    mu, logw, xm = enc(torch.from_numpy(tokens).cuda(), torch.tensor(lengths).cuda())
    (torch.sum(mu * torch.from_numpy(gmu).float().cuda()) + torch.sum(logw * torch.from_numpy(glw).float().cuda())).backward()
    sd = synthetic_text_encoder_state_dict(5)
    p = {k: torch.as_tensor(v).double().requires_grad_() for k, v in sd.items()}
    drop = ote.Dropouts(seed, p_drop, 0.5) if p_drop > 0 else None
    rmu, rlw, _ = ote.text_encoder(p, torch.from_numpy(tokens), torch.tensor(lengths), drop=drop)
    (torch.sum(rmu * torch.from_numpy(gmu)) + torch.sum(rlw * torch.from_numpy(glw))).backward()
    report(f"encoder train pass mu_x p={p_drop}", rel_err(mu.detach().cpu().numpy(), rmu.detach().numpy()), 1e-5)
    report(f"encoder train pass logw p={p_drop}", rel_err(logw.detach().cpu().numpy(), rlw.detach().numpy()), 1e-5)
    names = list(sd.keys())
    params = dict(enc.named_parameters())
    ours = {k: params[k].grad.detach().cpu().numpy().astype(np.float64) for k in names}
    refg = {k: p[k].grad.numpy() for k in names}
    gsq, gproj = grad_digest(ours, names)
    rsq, rproj = grad_digest(refg, names)
    rn = np.sqrt(rsq)
    err = np.maximum(np.abs(np.sqrt(gsq) - rn), np.abs(gproj - rproj)) / (rn + 1e-3 * rn.max())
    report(f"encoder train pass grad digests p={p_drop} (worst {names[int(err.argmax())]})", float(err.max()), 5e-5)
    worst = max(rel_err(ours[k], refg[k]) for k in names if np.abs(refg[k]).max() > 1e-3 * max(
        np.abs(v).max() for v in refg.values()))
    report(f"encoder train pass elementwise grads p={p_drop}", worst, 5e-5)


def test_compute_loss_speed_vs_torch_eager(mas_oracle):
    """Report (no gate) one GradTTS training step's loss + backward at the reference's training shape (params.py:
    batch 16, out_size 172 frames; ~6 s utterances of ~120-190 tokens) against torch eager autograd of the same
    objective on the same GPU (oracle/tts_loss.py in fp32 on CUDA: MIOpen convs, the MAS on the host as the
    reference runs it)."""
    import time
    from oracle import tts_loss
    rng = np.random.default_rng(5)
    B, Tx, out_size = 16, 190, 172
    x_lengths = rng.integers(120, Tx + 1, B)
    x_lengths[0] = Tx
    y_lengths = (x_lengths * rng.uniform(3.0, 4.0, B)).astype(np.int64)
    Ty = int(y_lengths.max())
    tokens = rng.integers(0, 149, (B, Tx)).astype(np.int64)
    y = (rng.standard_normal((B, 80, Ty)) * 1.5).astype(np.float32)
    for b in range(B):
        y[b, :, y_lengths[b]:] = 0
    m = make_gradtts().train()
    c = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    args = (c(tokens), c(x_lengths), c(y), c(y_lengths))

    def ours():
        m.zero_grad(set_to_none=True)
        random.seed(1)
        dur, prior, diff = m.compute_loss(*args, out_size=out_size)
        (dur + prior + diff).backward()

    ep = tts_loss.params(synthetic_text_encoder_state_dict(5), torch.float32, "cuda")
    dp = tts_loss.params(synthetic_state_dict(seed=0), torch.float32, "cuda")
    t = rng.uniform(1e-5, 1 - 1e-5, B).astype(np.float32)
    z = rng.standard_normal((B, 80, out_size)).astype(np.float32)
    offsets = [int(rng.integers(0, max(1, yl - out_size))) for yl in y_lengths]

    def eager():
        for v in list(ep.values()) + list(dp.values()):
            v.grad = None
        dur, prior, diff, _ = tts_loss.compute_loss(ep, dp, *args, offsets, out_size, c(t), c(z), mas_oracle,
                                                    dtype=torch.float32)
        (dur + prior + diff).backward()

    def timed(fn, n=5):
        fn(); fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    ms_ours, ms_eager = timed(ours), timed(eager)
    report(f"GradTTS.compute_loss + backward B={B} Tx<={Tx} Ty<={Ty} out_size={out_size}: ours {ms_ours:.2f} ms, "
           f"torch eager {ms_eager:.2f} ms; ratio eager/ours", ms_eager / ms_ours, 0.0, gate=False,
           ms_ours=ms_ours, ms_eager=ms_eager)


def test_optimizer_step_device_sync_matches_fresh_upload():
    """After optimizer steps the drop-ins hand the new parameters to the library on the device
    (gt_text_encoder_set_params_device / gt_decoder_set_params_device: copy + device repack, no host round trip).
    The next compute_loss + backward, a reverse-diffusion decode (inference images re-packed from the device block)
    and the encoder's inference pass must equal those of a fresh model loaded with the same state_dict (host upload),
    bit for bit."""
    g = load_golden("tts_loss_B2.npz")
    m = make_gradtts(int(g["seed_enc"]), int(g["seed_dec"])).eval()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        dur, prior, diff = run_fixture(m, g)
        (dur + prior + diff).backward()
        opt.step()
    m2 = make_gradtts(int(g["seed_enc"]), int(g["seed_dec"])).eval()
    m2.load_state_dict(m.state_dict())
    outs = []
    for mm in (m, m2):
        mm.zero_grad(set_to_none=True)
        losses = run_fixture(mm, g)
        sum(losses).backward()
        grads = [p.grad.detach().clone() for p in mm.parameters()]
        with torch.no_grad():
            tok = torch.from_numpy(g["tokens"]).cuda()
            mu_x, logw, _ = mm.encoder(tok, torch.from_numpy(g["x_lengths"]).cuda())
            torch.manual_seed(0)
            z = torch.randn(2, 80, 32, device="cuda")
            mask = torch.ones(2, 1, 32, device="cuda")
            y = mm.decoder(z, mask, torch.zeros_like(z), 3)
        outs.append(([float(v) for v in losses], grads, mu_x, logw, y))
    a, b = outs
    assert a[0] == b[0]
    assert all(torch.equal(x, y) for x, y in zip(a[1], b[1]))
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3]) and torch.equal(a[4], b[4])


def test_two_taped_forwards_before_backward():
    """Gradient accumulation: two compute_loss calls (two encoder tapes alive) and one backward of their sum give the
    gradients of two separate backward passes (the library's backward is stateless: each tape carries its own)."""
    g = load_golden("tts_loss_B2.npz")
    m = make_gradtts(int(g["seed_enc"]), int(g["seed_dec"])).eval()
    g2 = dict(g)
    g2["tokens"] = np.ascontiguousarray(g["tokens"][::-1])
    g2["x_lengths"] = np.ascontiguousarray(g["x_lengths"][::-1])
    g2["y"] = np.ascontiguousarray(g["y"][::-1])
    g2["y_lengths"] = np.ascontiguousarray(g["y_lengths"][::-1])
    m.zero_grad(set_to_none=True)
    l1 = sum(run_fixture(m, g))
    l2 = sum(run_fixture(m, g2))
    (l1 + l2).backward()
    together = [p.grad.detach().clone() for p in m.parameters()]
    m.zero_grad(set_to_none=True)
    sum(run_fixture(m, g)).backward()
    sum(run_fixture(m, g2)).backward()
    apart = [p.grad.detach().clone() for p in m.parameters()]
    for a, b in zip(together, apart):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


def _encoder_inputs(seed, lengths, n_vocab=149):
    rng = np.random.default_rng(seed)
    tokens = rng.integers(0, n_vocab, size=(len(lengths), max(lengths))).astype(np.int64)
    return torch.from_numpy(tokens).cuda(), torch.tensor(lengths).cuda()


def test_encoder_retain_graph_second_backward():
    """A second backward through the same graph (retain_graph=True) differentiates the same tape again and gives the
    same gradients, as the reference's autograd does (the tape stays alive until autograd frees the graph)."""
    enc = make_gradtts().encoder.eval()
    tokens, lengths = _encoder_inputs(9, [21, 13])
    mu, logw, _ = enc(tokens, lengths)
    loss = mu.square().sum() + logw.sum()
    loss.backward(retain_graph=True)
    g1 = [p.grad.detach().clone() for p in enc.parameters()]
    enc.zero_grad(set_to_none=True)
    loss.backward()
    g2 = [p.grad.detach().clone() for p in enc.parameters()]
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))


def test_encoder_backward_refuses_parameters_changed_on_device():
    """A device-side parameter update (gt_text_encoder_set_params_device, as after an optimizer step) between the
    taped forward and its backward: the tape holds activations of the old weights, so the backward must fail with
    GT_ERR_PARAM instead of returning silently wrong gradients."""
    from gradtts_amd import _lib
    from gradtts_amd.diffusion import _stream_ptr
    enc = make_gradtts().encoder.eval()
    tokens, lengths = _encoder_inputs(10, [17, 9])
    mu, logw, _ = enc(tokens, lengths)
    loss = mu.sum() + logw.sum()
    L = _lib.lib()
    h = enc._native()
    named = dict(enc.named_parameters())
    names = [L.gt_text_encoder_param_name(h, i).decode() for i in range(L.gt_text_encoder_num_params(h))]
    flat = torch.cat([named[n].detach().reshape(-1) for n in names]) * 1.01
    _lib.check(L.gt_text_encoder_set_params_device(h, flat.data_ptr(), flat.numel(), _stream_ptr(flat.device)),
               "gt_text_encoder_set_params_device")
    with pytest.raises(_lib.GradTTSError, match="parameters changed"):
        loss.backward()


def test_text_encoder_large_vocabulary_embedding_gradient():
    """n_vocab x C above the backward's 8 M-float partial buffer (C = 192: n_vocab > 43,690, e.g. a BPE vocabulary):
    the embedding gradient goes straight into the gradient buffer instead of past the partials. Checked elementwise
    on the rows of the tokens used (ids up to 44,999) against fp64 autograd through the oracle."""
    from oracle import text_encoder as ote
    from gradtts_amd.text_encoder import TextEncoder
    nv = 45000
    enc = TextEncoder(nv, 80, 192, 768, 256, 2, 6, 3, 0.1, 4)
    sd = synthetic_text_encoder_state_dict(5, n_vocab=nv)
    enc.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    enc = enc.cuda().eval()
    lengths = [19, 12]
    tokens, lens = _encoder_inputs(11, lengths, nv)
    tokens[0, :3] = torch.tensor([nv - 1, 43691, 0])
    mu, logw, _ = enc(tokens, lens)
    (mu.sum() + 0.5 * logw.sum()).backward()
    p = {k: torch.as_tensor(v).double().requires_grad_() for k, v in sd.items()}
    rmu, rlw, _ = ote.text_encoder(p, tokens.cpu(), lens.cpu())
    (rmu.sum() + 0.5 * rlw.sum()).backward()
    used = torch.unique(tokens.cpu()).numpy()
    ours = enc.emb.weight.grad.detach().cpu().numpy()[used]
    ref = p["emb.weight"].grad.numpy()[used]
    report("large-vocabulary embedding gradient (n_vocab 45000)", rel_err(ours, ref), 5e-5)
    unused = np.setdiff1d(np.arange(nv), used)
    assert not np.any(enc.emb.weight.grad.detach().cpu().numpy()[unused])
