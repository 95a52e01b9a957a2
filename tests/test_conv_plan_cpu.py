"""Launch planning of the ResNet convolutions (csrc/kernels/conv_gemm.hip conv_gemm_plan,
conv_gemm_wgrad_ppc), host-only: every ResNet-18 layer at the benchmark batch gets a
valid plan - tiles that divide the channels, K splits that cover K without empty splits,
the parity-class data gradient exactly for stride 2 - and the choices the sweep in
profiles/r1_resnet/conv_sweep.jsonl measured as best."""
import pytest
import torch

from ddp_amd import native

BF = torch.bfloat16


def resnet18_convs(B=32):
    out = [("stem", B, 224, 4, 64, 7, 2, 3), ("l1.3x3", B, 56, 64, 64, 3, 1, 1)]
    for i, (cin, cout, h) in enumerate(((64, 128, 56), (128, 256, 28), (256, 512, 14)), start=2):
        out += [(f"l{i}.3x3s2", B, h, cin, cout, 3, 2, 1), (f"l{i}.3x3", B, h // 2, cout, cout, 3, 1, 1),
                (f"l{i}.1x1s2", B, h, cin, cout, 1, 2, 0)]
    return out


def _shapes(N, H, Cin, Cout, K, s, p):
    OH = (H + 2 * p - K) // s + 1
    # geometry only: tiny meta tensors are enough (the planner reads sizes)
    x = torch.empty(N, H, H, Cin, dtype=BF)
    y = torch.empty(N, OH, OH, Cout, dtype=BF)
    return x, y, OH


@pytest.mark.parametrize("layer", resnet18_convs(), ids=lambda l: l[0])
def test_plans_are_valid(layer):
    C = native.require()
    name, N, H, Cin, Cout, K, s, p = layer
    x, y, OH = _shapes(N, H, Cin, Cout, K, s, p)
    bp, bc, splits, rows, par, halo = C.conv_gemm_plan(x, y, K, K, s, p, False)
    assert bp in (64, 128) and bc in (64, 128) and Cout % bc == 0 and par == 0
    nk = ((K * K + 7) // 8) if Cin == 4 else K * K * Cin // 32
    assert 1 <= splits <= min(8, nk)
    P = N * OH * OH
    # the halo-tile forward takes the stride-1 3x3 layers whose row-block grid fills the GPU
    # (56/28 wide: 128-pixel tiles, 14 wide: 64-pixel tiles; not the 7-wide layer4)
    assert halo == (1 if (K == 3 and s == 1 and H >= 14) else 0)
    if halo:
        R = bp // H
        assert splits <= Cin // 32 and (splits > 1 or rows == N * -(-H // R))
    elif splits == 1:
        assert rows == -(-P // bp)
    if Cin != 4:
        bp, bc, splits, _, par, halo = C.conv_gemm_plan(x, y, K, K, s, p, True)
        assert halo == (1 if (K == 3 and s == 1 and H >= 14) else 0)  # halo dgrad likewise
        assert bc in (64, 128) and Cin % bc == 0
        assert par == (1 if s == 2 else 0)
        assert splits >= 1
    ppc = C.conv_gemm_wgrad_ppc(x, y, K, K, s, p)
    # per-tap GEMM chunks: multiples of its 32-pixel K-step; halo wgrad (stride-1 3x3 layers
    # where the GEMM would run 64x64 tiles): whole output rows (whole images when stacked)
    halo_w = K == 3 and s == 1
    assert ppc >= 32 and (ppc % (OH * OH if OH < 28 else OH) == 0 if halo_w else ppc % 32 == 0)
    chunks = C.conv_gemm_wgrad_chunks(x, y, K, K, s, p, ppc)
    assert chunks * ppc >= P and (chunks - 1) * ppc < P


def test_plans_match_sweep_winners():
    """Spot checks against the measured best plans (profiles/r1_resnet/conv_sweep.jsonl)."""
    C = native.require()
    layers = {l[0]: l for l in resnet18_convs()}

    def plan(name, dgrad):
        _, N, H, Cin, Cout, K, s, p = layers[name]
        x, y, _ = _shapes(N, H, Cin, Cout, K, s, p)
        return C.conv_gemm_plan(x, y, K, K, s, p, dgrad)

    assert plan("l1.3x3", False)[5] == 1 and plan("l1.3x3", False)[2] == 1   # halo tile
    assert plan("l4.3x3", False)[5] == 0 and plan("l4.3x3", False)[2] == 8   # 7 wide: split 8 ways
    assert plan("l3.1x1s2", False)[:3] == (64, 64, 1)
    assert plan("l2.3x3s2", True)[:3] == (128, 64, 1) and plan("l2.3x3s2", True)[4] == 1
    assert plan("l4.1x1s2", True)[:3] == (64, 64, 1)
    # weight gradient: tap-fused halo kernel on every stride-1 3x3 layer (profiles/r2_halo_wgrad):
    # whole-row chunks, ~256 blocks of 64 co x 32 ci
    for name, ppc in (("l1.3x3", 14 * 56), ("l2.3x3", 28 * 28), ("l3.3x3", 56 * 14), ("l4.3x3", 112 * 7)):
        _, N, H, Cin, Cout, K, s, p = layers[name]
        x, y, _ = _shapes(N, H, Cin, Cout, K, s, p)
        got = C.conv_gemm_wgrad_ppc(x, y, K, K, s, p)
        assert got == ppc, (name, got)


def test_explicit_plan_overrides_and_bad_tiles():
    C = native.require()
    x, y, _ = _shapes(2, 14, 128, 256, 3, 1, 1)
    assert C.conv_gemm_plan(x, y, 3, 3, 1, 1, False, 64, 64, 3)[:3] == (64, 64, 3)
    assert C.conv_gemm_plan(x, y, 3, 3, 1, 1, False, 0, 0, 0, -1, 0)[5] == 0  # halo off on request
    x2, y2, _ = _shapes(2, 14, 128, 256, 3, 2, 1)
    assert C.conv_gemm_plan(x2, y2, 3, 3, 2, 1, True, 0, 0, 0, 0)[4] == 0  # parity off on request
    with pytest.raises(RuntimeError):
        C.conv_gemm_plan(x, y, 3, 3, 1, 1, False, 96, 0, 0)
