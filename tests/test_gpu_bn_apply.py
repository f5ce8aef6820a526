"""Block-tiled BatchNorm apply (csrc/bn_ops.hip bn_seg_apply_blk_f32_kernel).

Both applies -- scale / shift from the producer epilogue's fp64 sums, or from
a finalize's rows -- run block-tiled by default: a block owns up to 128 KB of
rows with their videos' scale / shift in LDS. Checked against the
per-thread-row kernels they replace (RNB_BN_APPLY_BLK=0) and against an fp64
reference: every channel width of R(2+1)D-34 (64 .. 1152, past the LDS
limit of 512), rows per clip from 49 (conv5) to 25088 (conv2), videos of
several clips, empty padding videos and bucket rows past the last video,
residual and ReLU, in place, and the indirect destination pointer.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _case(C, rpc, clips_per_video, pad_clips, seed=0):
    g = torch.Generator().manual_seed(seed)
    offs = [0]
    for n in clips_per_video:
        offs.append(offs[-1] + n)
    nclips = offs[-1] + pad_clips
    offs_pad = offs + [offs[-1]]                  # one empty padding video
    M = nclips * rpc
    y = (torch.randn((M, C), generator=g) * 3 + 1).to(DEV)
    res = torch.randn((M, C), generator=g).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.1).to(DEV)
    coffs = torch.tensor(offs_pad, dtype=torch.int32, device=DEV)
    nseg = len(offs_pad) - 1
    sums = torch.zeros((nseg, 2, C), dtype=torch.float64, device=DEV)
    for s in range(nseg):
        a, b = offs_pad[s] * rpc, offs_pad[s + 1] * rpc
        if b > a:
            yd = y[a:b].double()
            sums[s, 0] = yd.sum(0)
            sums[s, 1] = (yd * yd).sum(0)
    return y, res, gamma, beta, coffs, nseg, sums, M, offs_pad


def _ref(y, res, gamma, beta, offs, rpc, eps, relu, sums):
    z = torch.zeros_like(y, dtype=torch.float64)
    for s in range(len(offs) - 1):
        a, b = offs[s] * rpc, offs[s + 1] * rpc
        if b <= a:
            continue
        n = b - a
        mean = sums[s, 0] / n
        var = (sums[s, 1] / n - mean * mean).clamp(min=0)
        sc = gamma.double() / torch.sqrt(var + eps)
        z[a:b] = (y[a:b].double() - mean) * sc + beta.double()
        if res is not None:
            z[a:b] += res[a:b].double()
    if relu:
        z = z.clamp(min=0)
    last = offs[-1] * rpc
    z[last:] = 0
    return z


@pytest.mark.parametrize("C,rpc,videos,pad", [
    (64, 25088, [1, 1], 1),          # conv2 block output, 1-clip videos, a padding clip
    (64, 392, [3, 1, 2], 0),         # many videos per block
    (144, 784, [2, 1], 1),
    (256, 392, [1] * 9, 2),          # conv4: 9 one-clip videos + padding
    (512, 49, [1, 15, 1, 1], 1),     # conv5 rows per clip: blocks span several videos
    (1152, 49, [1, 2], 0),           # past the LDS scale / shift limit (per-item path)
])
@pytest.mark.parametrize("mode", ["sums", "ss"])
def test_blocked_apply_matches_rowwise_and_fp64(C, rpc, videos, pad, mode):
    from rnb_amd.ops.native import kernels
    k = kernels()
    eps = 1e-3
    y, res, gamma, beta, coffs, nseg, sums, M, offs = _case(C, rpc, videos, pad)
    stream = torch.cuda.current_stream().cuda_stream
    ss = None
    if mode == "ss":
        mean = torch.empty((nseg, C), device=DEV)
        var = torch.empty((nseg, C), device=DEV)
        ss = torch.empty((nseg, 2, C), device=DEV)
        k.bn_seg_ss_from_sums_f32(sums.data_ptr(), C, coffs.data_ptr(), nseg, rpc, C,
                                  gamma.data_ptr(), beta.data_ptr(), eps, mean.data_ptr(),
                                  var.data_ptr(), ss.data_ptr(), stream)
    outs = {}
    for blk in (0, 1):
        k.bn_set_apply_blk(bool(blk))
        for with_res in (False, True):
            z = torch.full_like(y, float("nan"))
            r = res if with_res else None
            if mode == "sums":
                k.bn_seg_apply_sums_f32(y.data_ptr(), z.data_ptr(), r.data_ptr() if r is not None
                                        else None, coffs.data_ptr(), nseg, rpc, sums.data_ptr(),
                                        C, gamma.data_ptr(), beta.data_ptr(), eps, 1, M, C, C, C,
                                        C if r is not None else 0, stream)
            else:
                k.bn_seg_apply_f32(y.data_ptr(), z.data_ptr(), r.data_ptr() if r is not None
                                   else None, coffs.data_ptr(), nseg, rpc, ss.data_ptr(), 1, M, C,
                                   C, C, C if r is not None else 0, stream)
            outs[(blk, with_res)] = z
    k.bn_set_apply_blk(True)
    torch.cuda.synchronize()
    for with_res in (False, True):
        a, b = outs[(0, with_res)], outs[(1, with_res)]
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-6), (C, rpc, with_res)
        ref = _ref(y, res if with_res else None, gamma, beta, offs, rpc, eps, True, sums)
        assert (b.double() - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()


def test_blocked_apply_in_place_and_indirect():
    """In place (z = y) and through a device-held destination pointer (the
    graphs that write a pipeline stage's output slot)."""
    from rnb_amd.ops.native import kernels
    k = kernels()
    C, rpc = 128, 784
    y, res, gamma, beta, coffs, nseg, sums, M, offs = _case(C, rpc, [2, 1, 1], 1, seed=3)
    stream = torch.cuda.current_stream().cuda_stream
    want = torch.empty_like(y)
    k.bn_seg_apply_sums_f32(y.data_ptr(), want.data_ptr(), res.data_ptr(), coffs.data_ptr(), nseg,
                            rpc, sums.data_ptr(), C, gamma.data_ptr(), beta.data_ptr(), 1e-3, 1, M,
                            C, C, C, C, stream)
    yi = y.clone()
    k.bn_seg_apply_sums_f32(yi.data_ptr(), yi.data_ptr(), res.data_ptr(), coffs.data_ptr(), nseg,
                            rpc, sums.data_ptr(), C, gamma.data_ptr(), beta.data_ptr(), 1e-3, 1, M,
                            C, C, C, C, stream)
    dst = torch.full_like(y, float("nan"))
    ind = torch.tensor([dst.data_ptr()], dtype=torch.int64, device=DEV)
    junk = torch.empty_like(y)
    k.bn_seg_apply_sums_f32(y.data_ptr(), junk.data_ptr(), res.data_ptr(), coffs.data_ptr(), nseg,
                            rpc, sums.data_ptr(), C, gamma.data_ptr(), beta.data_ptr(), 1e-3, 1, M,
                            C, C, C, C, stream, ind.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(yi, want)
    assert torch.equal(dst, want)
