"""End-to-end GPU tests: engine, graphs, fused serving path, IPC, tracer."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _engines(start, end, depth=18):
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    net = build_network(start, end, depth=depth, seed=3)
    return (R2P1DEngine(net, DEV, backend="hip"), R2P1DEngine(net, DEV, backend="torch"),
            R2P1DEngine(net, DEV, backend="module"))


@pytest.mark.parametrize("rng", [(1, 5), (1, 2), (3, 5), (2, 4)])
def test_engine_hip_matches_torch_plan(rng):
    hip, ref, mod = _engines(*rng)
    x = torch.randn(hip.input_shape(3), device=DEV).to(torch.bfloat16)
    if rng[0] == 1:
        x[..., 3:] = 0
    y = hip.forward(x).float()
    r = ref.forward(x).float()
    m = mod.forward(x).float()
    torch.cuda.synchronize()
    scale = r.abs().max().item()
    assert (y - r).abs().max().item() <= 3e-2 * scale + 3e-2
    # folded bf16 plan vs the unfolded fp32 nn.Module
    assert (r - m).abs().max().item() <= 5e-2 * scale + 5e-2


def test_r34_full_forward_close_to_module():
    hip, ref, mod = _engines(1, 5, depth=34)
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    x = SyntheticDecoder(DEV).decode(11, [0, 100, 200])
    y = hip.forward(x)
    m = mod.forward(x)
    torch.cuda.synchronize()
    rel = (y - m).abs().max().item() / m.abs().max().item()
    assert rel < 5e-2, rel
    assert torch.equal(y.argmax(1), m.argmax(1)) or rel < 1e-2


def test_graphed_engine_matches_eager():
    from rnb_amd.models.r2p1d.engine import GraphedEngine
    hip, _, _ = _engines(1, 5)
    ge = GraphedEngine(hip, max_clips=6, buckets=(1, 2, 4), autotune=False)
    for n in (1, 3, 6):
        x = torch.randn(hip.input_shape(n), device=DEV).to(torch.bfloat16)
        x[..., 3:] = 0
        a = ge(x).clone()
        b = hip.forward(x)
        torch.cuda.synchronize()
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-3)


def test_fused_serving_matches_stepwise():
    from rnb_amd.models.r2p1d.fused import FusedR2P1D
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    from rnb_amd.ops import video as vops
    f = FusedR2P1D(DEV, depth=18, replicas=2, max_clips=32, max_videos=4,
                   buckets=(4, 16, 32), autotune=False)
    videos = [(5, [0, 50]), (9, [3]), (12, list(range(0, 120, 8))), (20, [7])]
    ev, out, nvid = f.replicas[1].submit(videos)
    ev.synchronize()
    got = out.tolist()
    dec = SyntheticDecoder(DEV)
    want = []
    for vid, st in videos:
        logits = f.engine.forward(dec.decode(vid, st))
        want.append(int(logits.float().sum(0).argmax()))
    assert got == want


def test_autotune_picks_valid_config():
    hip, _, _ = _engines(1, 5)
    chosen = hip.autotune(2, reps=1)
    from rnb_amd.ops.native import kernels
    from rnb_amd.ops.conv import SPECIAL_NAMES
    assert all(0 <= c < len(kernels().configs) or c in SPECIAL_NAMES for c in chosen.values())
    # fused (2+1)D pairs: a conv21.hip variant or None (two-kernel path)
    assert hip.fused_choices and all(v in (None, 0, 1) for v in hip.fused_choices.values())


def _ipc_child(q_in, q_out):
    import torch
    from rnb_amd.ops import native
    rt = native.runtime()
    torch.cuda.set_device(0)
    handle, nbytes = q_in.get()
    ptr = rt.ipc_open_handle(handle)
    dst = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda:0")
    s = torch.cuda.current_stream()
    rt.memcpy_async(dst.data_ptr(), ptr, nbytes, s.cuda_stream)
    s.synchronize()
    q_out.put(dst.sum().item())
    rt.ipc_close_handle(ptr)


def test_hip_ipc_roundtrip_two_processes():
    import torch.multiprocessing as mp
    from rnb_amd.ops import native
    rt = native.runtime()
    torch.cuda.set_device(0)
    n = 1 << 12
    ptr = rt.ipc_malloc(n * 4)
    src = torch.arange(n, dtype=torch.float32, device=DEV)
    rt.memcpy_async(ptr, src.data_ptr(), n * 4, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=_ipc_child, args=(q_in, q_out))
    p.start()
    q_in.put((rt.ipc_get_handle(ptr), n * 4))
    total = q_out.get(timeout=120)
    p.join(60)
    rt.free(ptr)
    assert p.exitcode == 0
    assert total == float(n * (n - 1) // 2)


_TRACER_CHILD = r"""
import sys
sys.path.insert(0, %r)
from rnb_amd.profiling import tracer
tracer.initialize()            # must precede HIP runtime initialisation
import torch
from rnb_amd.models.r2p1d.model import build_network
from rnb_amd.models.r2p1d.engine import R2P1DEngine
dev = torch.device("cuda:0")
hip = R2P1DEngine(build_network(1, 5, depth=18), dev, backend="hip")
x = torch.zeros(hip.input_shape(1), device=dev, dtype=torch.bfloat16)
hip.forward(x)
torch.cuda.synchronize()
tracer.flush()
recs = tracer.report()
names = [r[0] for r in recs]
assert len(recs) >= 40, len(recs)
assert any("conv_igemm" in n for n in names), names[:5]
assert all(e >= s for _, s, e in recs)
print("TRACER_OK", len(recs))
"""


def test_tracer_reports_kernels():
    import subprocess
    import sys
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, "-c", _TRACER_CHILD % here],
                         capture_output=True, text=True, timeout=300)
    assert res.returncode == 0 and "TRACER_OK" in res.stdout, res.stdout + res.stderr


def test_native_libraries_loaded_from_tree():
    from rnb_amd.ops import native
    native.kernels()
    paths = native.loaded_paths()
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert any(p.startswith(here) for p in paths)


@pytest.mark.gpu
def test_amdsmi_vram_query():
    from rnb_amd.config import gpu_memory_used_bytes
    used = gpu_memory_used_bytes()
    assert used is not None and len(used) >= 1 and all(u >= 0 for u in used)


def test_batch_bn_mode_hip_matches_torch_and_module():
    """Reference training-mode BN numerics on the HIP kernels (eager, no graphs)."""
    from rnb_amd.models.r2p1d.model import build_network, build_engine
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    x = torch.randn(3, 3, 8, 112, 112, generator=torch.Generator().manual_seed(2)).to(DEV)
    mk = lambda b: R2P1DEngine(build_network(1, 5, depth=18, seed=4), DEV, backend=b,
                               bn_mode="batch")
    hip, tor, mod = mk("hip"), mk("torch"), mk("module")
    from rnb_amd.ops.video import ncdhw_to_ndhwc
    xb = ncdhw_to_ndhwc(x, 8)
    with torch.no_grad():
        a = hip.forward(xb).float()
        b = tor.forward(xb).float()
        m = mod.forward(x).float()
    torch.cuda.synchronize()
    scale = m.abs().max().item()
    e_hip, e_tor = (a - m).abs().max().item(), (b - m).abs().max().item()
    print("batch-BN max err vs fp32 module: hip %.4f torch-plan %.4f (scale %.3f)"
          % (e_hip, e_tor, scale))
    # both bf16 plans drift from the fp32 module by the same order (batch
    # statistics renormalise every layer, so bf16 rounding does not cancel)
    assert e_hip <= max(2.0 * e_tor, 3e-2 * scale)
    assert e_hip <= 8e-2 * scale
    eng = build_engine(DEV, depth=18, bn_mode="batch", backend="hip", dtype="bf16")
    assert isinstance(eng, R2P1DEngine) and eng.bn_mode == "batch"


def test_top1_agreement_512_clips_bf16_and_fp32_vs_fp32_module():
    """Verdict round 1 item 8: over 512 synthetic clips, the argmax of the
    bf16 and fp32 HIP engines must agree with the fp32 nn.Module on >= 99 %
    of the clips (fp32: all of them up to exact near-ties)."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    dev = torch.device("cuda:0")
    net = build_network(1, 5, depth=34, seed=3)
    mod = R2P1DEngine(net, dev, backend="module", dtype="fp32")
    e32 = R2P1DEngine(net, dev, backend="hip", dtype="fp32")
    e16 = R2P1DEngine(net, dev, backend="hip", dtype="bf16")
    dec = SyntheticDecoder(dev, dtype=torch.float32)
    agree16 = agree32 = total = 0
    with torch.no_grad():
        for b in range(8):                              # 8 x 64 = 512 clips
            x = torch.cat([dec.decode(1000 * b + v, [0, 20, 40, 60, 80, 100, 120, 140])
                           for v in range(8)])
            ref = mod.forward(x).argmax(1)
            a32 = e32.forward(x).argmax(1)
            x16 = torch.zeros(x.shape[:4] + (8,), dtype=torch.bfloat16, device=dev)
            x16[..., :3] = x[..., :3].to(torch.bfloat16)
            a16 = e16.forward(x16).argmax(1)
            agree32 += int((a32 == ref).sum())
            agree16 += int((a16 == ref).sum())
            total += x.shape[0]
    torch.cuda.synchronize()
    print("top-1 agreement over %d clips: fp32 %.4f bf16 %.4f"
          % (total, agree32 / total, agree16 / total))
    assert total == 512
    assert agree32 / total >= 0.99
    assert agree16 / total >= 0.99


def test_top1_agreement_batch_bn_graphed_per_video_vs_module():
    """The headline numerics: fp32 R(2+1)D-34 with
    training-mode BatchNorm (per-video batch statistics) through the bucket
    HIP graphs, 224 videos (200 one-clip + 24 fifteen-clip, 560 clips) packed
    into multi-video calls of <= 128 clips, against the fp32 nn.Module run
    once per video as the reference runs it. Top-1 agreement per clip >= 99 %
    and the logits' max error relative to the logit scale <= 5e-4: both sides
    are fp32 with different summation orders, and 36 batch-statistics BNs
    (1-clip videos: as few as 49 values per channel at conv5) amplify the
    ~1e-6 per-conv differences; test_batch_bn_fp32_error_vs_fp64 shows the
    HIP path is as close to an fp64 forward as PyTorch's fp32 module is."""
    from rnb_amd.models.r2p1d.model import build_engine, build_network
    from rnb_amd.models.r2p1d.engine import GraphedEngine, R2P1DEngine
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    import random
    dev = torch.device("cuda:0")
    g = build_engine(dev, depth=34, seed=11, bn_mode="batch", dtype="fp32", max_clips=128,
                     autotune=False)
    assert isinstance(g, GraphedEngine) and g.batch_bn
    mod = R2P1DEngine(build_network(1, 5, depth=34, seed=11), dev, backend="module",
                      bn_mode="batch", dtype="fp32")
    dec = SyntheticDecoder(dev, dtype=torch.float32)
    rng = random.Random(5)
    counts = [1] * 200 + [15] * 24
    rng.shuffle(counts)
    videos = [(v, sorted(rng.sample(range(0, 240), n))) for v, n in enumerate(counts)]
    batches, cur, ncl = [], [], 0
    for v in videos:
        if ncl + len(v[1]) > 128:
            batches.append(cur)
            cur, ncl = [], 0
        cur.append(v)
        ncl += len(v[1])
    batches.append(cur)
    agree = total = 0
    worst = 0.0
    with torch.no_grad():
        for b in batches:
            xs = [dec.decode(1000 + vid, starts) for vid, starts in b]
            offs = [0]
            for x in xs:
                offs.append(offs[-1] + x.shape[0])
            y = g.forward(torch.cat(xs), clip_offsets=offs).clone()
            ref = torch.cat([mod.forward(x) for x in xs])
            agree += int((y.argmax(1) == ref.argmax(1)).sum())
            total += y.shape[0]
            worst = max(worst, (y - ref).abs().max().item() / ref.abs().max().item())
    torch.cuda.synchronize()
    print("batch-BN graphed vs per-video module: %d calls, %d clips, top-1 %.4f, "
          "max rel err %.2e" % (len(batches), total, agree / total, worst))
    assert total == 560
    assert agree / total >= 0.99
    assert worst <= 5e-4, worst


def test_batch_bn_fp32_error_vs_fp64():
    """Error analysis behind the 5e-4 bound above: R(2+1)D-34 with per-video
    batch-statistics BN, three videos (1 + 1 + 3 clips) in one graphed call,
    against the same network in fp64 on the CPU (one video per forward). The
    HIP fp32 path (MFMA / split-bf16 Winograd, fp64 BN statistics) must be at
    least as close to fp64 as PyTorch's own fp32 module (MIOpen) is, within a
    factor 3."""
    import copy
    from rnb_amd.models.r2p1d.model import build_engine, build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    from rnb_amd.ops.video import ndhwc_to_ncdhw
    dev = torch.device("cuda:0")
    g = build_engine(dev, depth=34, seed=11, bn_mode="batch", dtype="fp32", max_clips=8,
                     buckets=[5, 8], autotune=False)
    net = build_network(1, 5, depth=34, seed=11)
    mod = R2P1DEngine(copy.deepcopy(net), dev, backend="module", bn_mode="batch",
                      dtype="fp32")
    net64 = copy.deepcopy(net).double().train()
    dec = SyntheticDecoder(dev, dtype=torch.float32)
    xs = [dec.decode(21, [30]), dec.decode(22, [100]), dec.decode(23, [0, 90, 180])]
    offs = [0, 1, 2, 5]
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    with torch.no_grad():
        y = g.forward(torch.cat(xs), clip_offsets=offs).double().cpu()
        ym = torch.cat([mod.forward(x) for x in xs]).double().cpu()
        y64 = torch.cat([net64(ndhwc_to_ncdhw(x, 3).double().cpu()) for x in xs])
    scale = y64.abs().max().item()
    e_hip = (y - y64).abs().max().item() / scale
    e_mod = (ym - y64).abs().max().item() / scale
    print("batch-BN fp32 vs fp64: HIP %.2e, PyTorch fp32 module %.2e" % (e_hip, e_mod))
    assert e_hip <= 3 * e_mod + 1e-6, (e_hip, e_mod)


def test_runner_lanes_match_one_lane():
    """R2P1DRunner(lanes=2): calls alternate over two graphed engines on two
    streams (inputs pulled on the caller's stream, outputs complete on
    ``completion_event()``); every output equals the one-lane runner's."""
    from rnb_amd.models.r2p1d.model import R2P1DRunner
    kw = dict(depth=10, bn_mode="batch", dtype="fp32", warmup=0, max_clips=4,
              bucket_step=1, autotune=False)
    one = R2P1DRunner(DEV, lanes=1, **kw)
    two = R2P1DRunner(DEV, lanes=2, **kw)
    assert two.lanes == 2 and two.inflight_calls() == 1
    g = torch.Generator(device=DEV).manual_seed(5)
    xs = [torch.randn(one.input_shape()[0][1:], device=DEV, generator=g)
          .unsqueeze(0).repeat(n, 1, 1, 1, 1) * (1 + 0.1 * i)
          for i, n in enumerate((1, 3, 2, 4, 1, 2))]
    outs = {}
    for name, r in (("one", one), ("two", two)):
        cur = torch.cuda.current_stream(DEV)
        res = []
        for x in xs:
            dst = r.gather_buffers(x.shape[0])[0]
            dst[:x.shape[0]].copy_(x)
            y = r((dst[:x.shape[0]],), None, None)[0][0]
            ev = r.completion_event()
            if ev is not None:
                cur.wait_event(ev)
            res.append(y.clone())
        torch.cuda.synchronize()
        outs[name] = res
    for a, b in zip(outs["one"], outs["two"]):
        assert torch.equal(a, b)


def test_batched_running_update_matches_per_bn_kernels(monkeypatch):
    """Calls of > 32 videos defer every BatchNorm's running update to one
    batched kernel at the end of the forward (RNB_BN_BATCH_RUNNING, default
    on): outputs and running statistics must equal the per-BN kernels'."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    g = torch.Generator().manual_seed(4)
    n = 40
    x = torch.randn((n, 2, 14, 14, 256), generator=g).to(DEV)
    offs = list(range(n + 1))                        # 40 one-clip videos
    outs, runs = [], []
    for flag in ("0", "1"):
        monkeypatch.setenv("RNB_BN_BATCH_RUNNING", flag)
        eng = R2P1DEngine(build_network(5, 5, depth=18, seed=2), DEV, backend="hip",
                          bn_mode="batch", dtype=torch.float32)
        for _ in range(2):
            y = eng.forward(x, clip_offsets=offs)
        torch.cuda.synchronize()
        outs.append(y.cpu())
        runs.append([(op.bn.running_mean.cpu(), op.bn.running_var.cpu())
                     for op in eng.ops if op.bn is not None])
    assert torch.equal(outs[0], outs[1])
    assert len(runs[0]) == len(runs[1]) > 0
    for (m0, v0), (m1, v1) in zip(runs[0], runs[1]):
        assert torch.allclose(m0, m1, rtol=1e-6, atol=1e-7)
        assert torch.allclose(v0, v1, rtol=1e-6, atol=1e-7)
        assert not torch.equal(v0, torch.ones_like(v0))    # updated at all


@pytest.mark.parametrize("env", ["RNB_BN_APPLY_SUMS", "RNB_BN_SS_ONLY"])
@pytest.mark.parametrize("n,per_video", [(40, 1), (6, 2)])
def test_apply_from_sums_matches_finalize_path(monkeypatch, n, per_video, env):
    """Block-output BatchNorms apply their scale / shift straight from the
    producer epilogue's sums (no finalize dispatch, RNB_BN_APPLY_SUMS), and
    the deferred BatchNorms' finalize computes scale / shift only
    (RNB_BN_SS_ONLY), both defaults: the batched running update walks the sums
    afterwards. Outputs bit-identical to the finalize paths, running
    statistics equal to theirs (in-order walk up to 16 videos, closed form
    above), the epilogue sums re-armed to zero for the next call."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    g = torch.Generator().manual_seed(5)
    x = torch.randn((n, 4, 28, 28, 128), generator=g).to(DEV)
    offs = list(range(0, n + 1, per_video))
    outs, runs = [], []
    for flag in ("0", "1"):
        monkeypatch.setenv(env, flag)
        eng = R2P1DEngine(build_network(4, 5, depth=18, seed=2), DEV, backend="hip",
                          bn_mode="batch", dtype=torch.float32)
        for _ in range(2):
            y = eng.forward(x, clip_offsets=offs)
        torch.cuda.synchronize()
        outs.append(y.cpu())
        runs.append([(op.bn.running_mean.cpu(), op.bn.running_var.cpu())
                     for op in eng.ops if op.bn is not None])
        for op in eng.ops:
            s = getattr(op.bn, "_esums", None) if op.bn is not None else None
            if s is not None:
                assert float(s.abs().sum()) == 0.0, "epilogue sums must be re-armed"
    assert torch.equal(outs[0], outs[1])
    for (m0, v0), (m1, v1) in zip(runs[0], runs[1]):
        assert torch.allclose(m0, m1, rtol=1e-6, atol=1e-7)
        assert torch.allclose(v0, v1, rtol=1e-6, atol=1e-7)
