"""modules.lstm.LSTM: the torch.nn.LSTM drop-in for the MD-VAE's `rnn: !new:torch.nn.LSTM`
(ref:src/models/MD_VAE/model.yaml:78-83: 2 layers, 512 units, unidirectional, batch_first,
dropout 0.15), multi-layer with train-mode dropout, against the oracle's explicit loop
(oracle/md_cpu.uni_lstm) with the Philox masks replayed on the host: output, (h_n, c_n) and the
gradients of sum(output * cot) with respect to the input and every parameter."""
import pytest
import torch

from gpu_utils import need_gpu, norm_rel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec,tol_out,tol_grad,H", [("fp32", 1e-5, 1e-4, 512), ("bf16", 1e-2, 3e-2, 512),
                                                     ("fp32", 1e-5, 1e-4, 1024)])
def test_md_vae_rnn_dropin_matches_oracle(prec, tol_out, tol_grad, H):
    """H = 1024 in fp32 runs the stepwise BPTT (nn.LSTM has no width limit)."""
    need_gpu()
    from mlvae_hip import ops
    from modules.lstm import LSTM
    from oracle import md_cpu as M
    from philox_np import dropout_mask
    B, T, I, L, p = 6, 40, 96, 2, 0.15
    torch.manual_seed(3)
    rnn = LSTM(input_size=I, hidden_size=H, num_layers=L, batch_first=True, dropout=p)
    assert isinstance(rnn, torch.nn.LSTM)
    params = {f"rnn.{k}": v.detach().clone().double().requires_grad_(True) for k, v in rnn.named_parameters()}
    x = torch.randn(B, T, I)
    cot = torch.randn(B, T, H)
    rnn = rnn.cuda().train()
    xd = x.cuda().requires_grad_(True)
    seed = 1234567
    prev = ops.get_precision()
    ops.set_precision(prec)
    try:
        out, (hn, cn) = ops.lstm_full(xd, rnn, True, seed=seed)
        (out * cot.cuda()).sum().backward()
    finally:
        ops.set_precision(prev)
    torch.cuda.synchronize()
    s0 = (seed * 1000003 + 0) & ((1 << 63) - 1)     # ops.LSTMFn's key of layer 0's dropout
    masks = [torch.from_numpy(dropout_mask(s0, B * T * H, p)).view(B, T, H).double()]
    xr = x.double().requires_grad_(True)
    ref = M.uni_lstm(params, xr, L, prefix="rnn.", dropout_masks=masks)
    (ref * cot.double()).sum().backward()
    assert norm_rel(out, ref) < tol_out
    assert norm_rel(hn[-1], ref[:, -1]) < tol_out          # last layer's h at t = T-1
    assert hn.shape == cn.shape == (L, B, H)
    errs = {k: norm_rel(v.grad, params[f"rnn.{k}"].grad) for k, v in rnn.named_parameters()}
    errs["x"] = norm_rel(xd.grad, xr.grad)
    print(f"\n[rnn drop-in {prec}] out {norm_rel(out, ref):.2e} " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    for k, v in errs.items():
        assert v < tol_grad, (k, v)


def test_rnn_dropin_module_forward_and_state_dict():
    need_gpu()
    from modules.lstm import LSTM
    torch.manual_seed(4)
    ref = torch.nn.LSTM(32, 64, num_layers=2, batch_first=True)
    mine = LSTM(32, 64, num_layers=2, batch_first=True)
    mine.load_state_dict(ref.state_dict())                    # the same keys and shapes
    assert list(mine.state_dict()) == list(ref.state_dict())
    x = torch.randn(3, 17, 32)
    mine = mine.cuda().eval()
    with torch.no_grad():
        o, (h, c) = mine(x.cuda())
        ro, (rh, rc) = ref.double()(x.double())
    from mlvae_hip import ops
    tol = 1e-5 if ops.get_precision() == "fp32" else 1e-2
    assert norm_rel(o, ro) < tol and norm_rel(h, rh) < tol and norm_rel(c, rc) < tol


def test_rnn_dropin_gradient_through_h_n_and_c_n():
    """h_n backpropagates as in nn.LSTM (its gradient joins each layer's output
    gradient at the last step, bidirectional included); a gradient through c_n is refused
    loudly instead of being dropped."""
    need_gpu()
    from mlvae_hip import ops
    torch.manual_seed(6)
    ref = torch.nn.LSTM(24, 32, num_layers=2, batch_first=True, bidirectional=True).double()
    mine = torch.nn.LSTM(24, 32, num_layers=2, batch_first=True, bidirectional=True)
    mine.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    mine = mine.cuda().eval()
    x = torch.randn(3, 11, 24)
    cot_o, cot_h = torch.randn(3, 11, 64), torch.randn(4, 3, 32)
    prev = ops.get_precision()
    ops.set_precision("fp32")
    try:
        xd = x.cuda().requires_grad_(True)
        o, hn, cn = ops.LSTMFn.apply(xd, 32, 2, 2, 0.0, 0, *[p for p in mine.parameters()])
        ((o * cot_o.cuda()).sum() + (hn * cot_h.cuda()).sum()).backward()
        xr = x.double().requires_grad_(True)
        ro, (rh, _) = ref(xr)
        ((ro * cot_o.double()).sum() + (rh * cot_h.double()).sum()).backward()
        assert norm_rel(xd.grad, xr.grad) < 1e-5
        for (k, a), (_, b) in zip(mine.named_parameters(), ref.named_parameters()):
            assert norm_rel(a.grad, b.grad) < 1e-5, k
        # only h_n used: the output's gradient arrives as None
        xd2 = x.cuda().requires_grad_(True)
        _, hn2, _ = ops.LSTMFn.apply(xd2, 32, 2, 2, 0.0, 0, *[p for p in mine.parameters()])
        hn2.sum().backward()
        assert torch.isfinite(xd2.grad).all()
        xd3 = x.cuda().requires_grad_(True)
        _, _, cn3 = ops.LSTMFn.apply(xd3, 32, 2, 2, 0.0, 0, *[p for p in mine.parameters()])
        with pytest.raises(NotImplementedError, match="c_n"):
            cn3.sum().backward()
    finally:
        ops.set_precision(prev)
