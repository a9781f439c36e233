"""Debug probe of the fp8 weight gradient in the engine: two fp8 steps at the c5 shard size, then
dW_ih_l1 recomputed from the engine's own e4m3 dG / layer input (fp64 on the host) against the
engine's gradient and the scales it used.  usage: python tools/dbg_fp8w.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-vae_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mlvae_hip.engine import VAEConfig, VAEEngine  # noqa: E402
from oracle import vae_cpu as O  # noqa: E402


def main():
    F, E, Z, H, L, C, B, T = 80, 64, 32, 512, 2, 64, 64, 500
    cfg = VAEConfig(F=F, E=E, Z=Z, H=H, L=L, C=C, dropout=0.15, prec="bf16", fp8=True)
    params = O.init_params(F, E, Z, H, L, C, seed=810)
    g = torch.Generator().manual_seed(810)
    eng = VAEEngine(cfg, params=params, seed=810)
    lens = torch.linspace(0.6, 1.0, B)
    for st in range(2):
        eng.train_step(torch.randn(B, T, F, generator=g).cuda(), lens.cuda())
        torch.cuda.synchronize()
        eng.check_errors()
    w = eng.work(B, T)
    N = B * T
    print("g8", eng.g8[1].tolist(), "g8w", eng.g8w[1].tolist(), "x8s", eng.x8s.tolist(), "w8s", eng.w8s[1].tolist())
    dG8 = w.dG8[1].view(torch.float8_e4m3fn).view(N, 8 * H).cpu().double()
    X8 = w.X8[1].view(torch.float8_e4m3fn).view(N, 2 * H).cpu().double()
    print("dG8 finite", bool(torch.isfinite(dG8).all()), "absmax", dG8.abs().max().item(),
          "X8 finite", bool(torch.isfinite(X8).all()), "absmax", X8.abs().max().item())
    ref = (dG8.t() @ X8) * eng.g8w[1][1].item()
    got = torch.cat([eng.view("decoder.rnn.weight_ih_l1", eng.grad), eng.view("decoder.rnn.weight_ih_l1_reverse",
                                                                             eng.grad)]).cpu().double()
    print("got absmax", got.abs().max().item(), "ref absmax", ref.abs().max().item())
    from mlvae_hip._lib import check, lib
    l = lib()
    C = torch.empty(8 * H, 2 * H, device="cuda")
    nb = l.mlvae_gemm_fp8_tn_workspace_size(8 * H, 2 * H, N)
    ws = torch.empty(nb // 4 + 1, device="cuda")
    check(l.mlvae_gemm_fp8_tn(8 * H, 2 * H, N, w.dG8[1].data_ptr(), 8 * H, w.X8[1].data_ptr(), 2 * H, C.data_ptr(), 2 * H,
                              eng.g8w[1].data_ptr() + 4, ws.data_ptr(), nb, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    Cd = C.cpu().double()
    print("direct call rel", ((Cd - ref).norm() / ref.norm()).item(), "absmax", Cd.abs().max().item())
    print("grad W_ih_l1: got norm", got.norm().item(), "ref norm", ref.norm().item(),
          "rel", ((got - ref).norm() / ref.norm()).item(), "finite", bool(torch.isfinite(got).all()))
    dGb = w.dGb[1].view(N, 8 * H).cpu().double()
    xin = w.layer_in[1][1]
    print("bf16 dG vs dG8/q rel", ((dGb - dG8 / eng.g8[1][0].item()).norm() / dGb.norm()).item())
    if xin is not None:
        xb = xin.view(N, 2 * H).cpu().double()
        print("bf16 x vs X8/xs rel", ((xb - X8 / eng.x8s[0].item()).norm() / xb.norm()).item())
        refb = dGb.t() @ xb
        print("bf16-operand dW vs engine rel", ((got - refb).norm() / refb.norm()).item())


if __name__ == "__main__":
    main()
