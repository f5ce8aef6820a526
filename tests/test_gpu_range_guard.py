"""h3 range guard (ops/conv_f32.RangeGuard; round-4 advice).

The h3 kernels scale activations by 2^6 before the fp16 hi/lo split, so an
input with |x| >= ~1024 would overflow fp16. The kernels flag any non-finite
output value into a host-coherent word, and the engine re-runs such a call on
full-range kernels. Checks: inputs of magnitude 2^11 - 2^14 trip the guard on
every h3 kernel family (direct, split-K, row band, temporal band) while 2^9
does not; the full-range configs stay within 1e-5 of an fp64 conv at those
magnitudes; a graphed batch-BN engine whose convs are forced onto h3 configs
re-runs a tripped call and then matches an fp64 module forward.
"""
import pytest
import torch

from test_gpu_f32 import DEV, _layer, _ref64

pytestmark = pytest.mark.gpu


def _scaled_input(n, thw, cin_p, cin, amp, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((n,) + thw + (cin_p,), generator=g)
    x = x / x.abs().max() * amp            # max |x| == amp
    x[..., cin:] = 0
    return x.to(DEV)


def _family_cases():
    from rnb_amd.ops.conv_f32 import H3D_BASE, H3K_BASE, H3R_BASE, H3T_BASE
    return [
        ("direct", (64, 144, (1, 3, 3), (1, 2, 2), (0, 1, 1)), (2, 14, 14), H3D_BASE + 2),
        ("splitk", (256, 256, (1, 3, 3), (1, 1, 1), (0, 1, 1)), (1, 7, 7), H3K_BASE + 0),
        ("rowband", (64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1)), (2, 14, 14), H3R_BASE + 7),
        ("temporal", (144, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0)), (8, 7, 7), H3T_BASE + 0),
    ]


@pytest.mark.parametrize("fam", range(4))
def test_range_guard_trips_on_overflow_and_full_range_is_exact(fam):
    from rnb_amd.ops.conv_f32 import RangeGuard, full_range, is_h3
    name, (cin, cout, k, s, p), thw, cid = _family_cases()[fam]
    layer = _layer(cin, cout, k, s, p)
    guard = RangeGuard()
    guard.activate()
    try:
        # in range: 2^9 * 2^6 = 32768 < 65504
        x = _scaled_input(2, thw, layer.geom.cin_p, cin, 2.0 ** 9)
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        assert not guard.tripped(), name
        ref = _ref64(layer, x)
        err = (y[..., :cout].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item(), (name, err)
        for lg in (11, 12, 13, 14):
            x = _scaled_input(2, thw, layer.geom.cin_p, cin, 2.0 ** lg, seed=lg)
            guard.reset()
            layer.forward_hip(x, config=cid)
            torch.cuda.synchronize()
            assert guard.tripped(), (name, lg)
            guard.reset()
            with full_range():
                fr = layer.config_for(x.shape)
                assert not is_h3(fr)
                y = layer.forward_hip(x)
            torch.cuda.synchronize()
            assert not guard.tripped()
            ref = _ref64(layer, x)
            err = (y[..., :cout].double().cpu() - ref).abs().max().item()
            assert err <= 1e-5 * ref.abs().max().item(), (name, lg, fr, err)
    finally:
        from rnb_amd.ops.native import kernels
        kernels().h3_set_range_flag(0)


def test_graphed_engine_reruns_tripped_call(monkeypatch):
    """R(2+1)D-34 layers 4-5 (input 128 x 4 x 28 x 28), training-mode BN, graphed, every conv forced onto
    an h3 config: an input of magnitude 2^13 trips the guard in the replay,
    range_fallback recomputes the call on full-range kernels, and the logits
    match an fp64 module forward (BN makes them invariant to the input scale,
    so they are O(1))."""
    from rnb_amd.models.r2p1d.engine import GraphedEngine, R2P1DEngine
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.ops import conv_f32
    from rnb_amd.ops.conv_f32 import ConvLayerF32, is_h3, is_h3k
    from rnb_amd.ops.video import ndhwc_to_ncdhw

    orig = ConvLayerF32._config_for

    def forced(self, x_shape):
        if conv_f32._FULL_RANGE[0]:
            return orig(self, x_shape)
        c = [i for i in self.candidates(x_shape) if is_h3(i) and not is_h3k(i)]
        if self.tune_with_affine:
            c = [i for i in c if self.affine_ok(i, x_shape)] or c
        return c[0]
    monkeypatch.setattr(ConvLayerF32, "_config_for", forced)

    net = build_network(4, 5, depth=34, seed=3)
    eng = R2P1DEngine(net, DEV, backend="hip", bn_mode="batch", dtype=torch.float32)
    assert eng.range_guard is not None
    geng = GraphedEngine(eng, 2, buckets=(2,), autotune=False, warmup=1)
    geng.prepare()
    n = 2
    x = _scaled_input(n, (4, 28, 28), eng.in_channels_p, 128, 2.0 ** 13, seed=5)
    static_in, _ = geng.input_buffer(n)
    static_in[:n].copy_(x)
    y = geng.replay(n)
    torch.cuda.synchronize()
    assert eng.range_guard.tripped()
    assert geng.range_fallback()
    torch.cuda.synchronize()
    assert not eng.range_guard.tripped()
    assert eng.range_guard.fallbacks == 1
    ref_net = build_network(4, 5, depth=34, seed=3).double().train()
    with torch.no_grad():
        ref = ref_net(ndhwc_to_ncdhw(x, 128).double().cpu())
    got = y.double().cpu()
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item(), (err, ref.abs().max().item())
    # the same input at 2^8 stays on the h3 graph: no fallback
    static_in[:n].copy_(x / 32)
    geng.replay(n)
    torch.cuda.synchronize()
    assert not eng.range_guard.tripped()
    assert not geng.range_fallback()


def test_bucket_padding_rows_do_not_trip_the_guard(monkeypatch):
    """A replay of n clips in a larger bucket computes the padding clips too.
    Their BatchNorm segment is empty: its scale / shift are 0 and the apply
    pass zeroes rows outside every segment, so padding rows stay bounded
    through all 72 convs of R(2+1)D-34 (round 5: they grew to inf through
    gamma / sqrt(eps) scales and tripped the guard on every padded call)."""
    from rnb_amd.models.r2p1d.engine import GraphedEngine, R2P1DEngine
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.ops import conv_f32
    from rnb_amd.ops.conv_f32 import ConvLayerF32, is_h3, is_h3k

    orig = ConvLayerF32._config_for

    def forced(self, x_shape):
        if conv_f32._FULL_RANGE[0]:
            return orig(self, x_shape)
        c = [i for i in self.candidates(x_shape) if is_h3(i) and not is_h3k(i)]
        if self.tune_with_affine:
            c = [i for i in c if self.affine_ok(i, x_shape)] or c
        return c[0] if c else orig(self, x_shape)
    monkeypatch.setattr(ConvLayerF32, "_config_for", forced)

    net = build_network(1, 5, depth=34, seed=1)
    eng = R2P1DEngine(net, DEV, backend="hip", bn_mode="batch", dtype=torch.float32)
    geng = GraphedEngine(eng, 4, buckets=(4,), autotune=False)
    geng.prepare()
    static_in, _ = geng.input_buffer(1)
    g = torch.Generator().manual_seed(0)
    static_in.copy_((torch.randn(static_in.shape, generator=g) * 3).to(DEV))
    for n, offs in ((1, None), (2, [0, 1, 2]), (3, None)):
        y = geng.replay(n, clip_offsets=offs)
        torch.cuda.synchronize()
        assert not eng.range_guard.tripped(), n
        assert torch.isfinite(y).all()


def test_engine_uses_h3_reflects_its_picks():
    """R2P1DEngine.uses_h3 (which decides whether a range-guarded non-final
    pipeline stage must synchronise each call): true after a
    forward that picked h3 configs, false once no conv holds an h3 pick."""
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.ops.conv_f32 import H3D_BASE
    eng = R2P1DEngine(build_network(1, 2, depth=18, seed=0), DEV, backend="hip",
                      bn_mode="batch", dtype=torch.float32)
    x = torch.randn((2, 8, 112, 112, 4), device=DEV)
    x[..., 3:] = 0
    for layer in eng.conv_layers():
        layer._config.clear()
    eng.forward(x, clip_offsets=[0, 2])
    torch.cuda.synchronize()
    for layer in eng.conv_layers():
        for k in list(layer._config):
            layer._config[k] = H3D_BASE           # force an h3 pick
    assert eng.uses_h3()
    for layer in eng.conv_layers():
        for k in list(layer._config):
            layer._config[k] = 0                  # fp32-MFMA direct config
    assert not eng.uses_h3()
