"""CPU check of the h3 Winograd kernel's weight image (ops/conv_f32.h3w_weights):
every (chunk, channel block, GEMM position, row, channel quad) entry holds the
fp16 hi / lo split of U = G g G^T * 2^sw at the chunk slot the kernel reads
(csrc/conv_h3w.hip h3w_swz), with hi + lo within 2^-22 of the fp64 value."""
import torch

from rnb_amd.ops.conv_f32 import _WINO_G, _WINO_SWZ, H3_W_TOP_LOG2, h3w_weights


def test_h3w_weight_image_roundtrip():
    g = torch.Generator().manual_seed(0)
    co, ci, cin_p, tc = 150, 40, 48, 3
    w = torch.randn((co, ci, 1, 3, 3), generator=g)
    u, sw = h3w_weights(w, cin_p, co, tc)
    ct = 16 * tc
    nb = (co + ct - 1) // ct
    assert u.dtype == torch.int16 and tuple(u.shape) == (cin_p // 16, nb, 16, ct, 4, 8)
    G = torch.tensor(_WINO_G, dtype=torch.float64)
    ref = torch.einsum("ik,ockl,jl->ocij", G, w.double().reshape(co, ci, 3, 3), G).reshape(co, ci, 16)
    full = torch.zeros(nb * ct, cin_p, 16, dtype=torch.float64)
    full[:co, :ci] = ref * 2.0 ** sw
    assert 2.0 ** H3_W_TOP_LOG2 <= full.abs().max() < 2.0 ** (H3_W_TOP_LOG2 + 1)
    h = u.view(torch.float16).double()
    rec = torch.zeros_like(full)
    for row in range(ct):
        s = _WINO_SWZ[(row % 16) >> 2]
        for q in range(4):
            chunk = h[:, :, :, row, q ^ s, :]                 # [ci/16, nb, 16x, 8]
            val = chunk[..., :4] + chunk[..., 4:]             # hi + lo per channel
            for b in range(nb):
                # [ci/16, 16x, 4 ch] -> channels 16 c + 4 q + i
                v = val[:, b].permute(0, 2, 1)                # [ci/16, 4, 16x]
                for c16 in range(cin_p // 16):
                    rec[b * ct + row, c16 * 16 + 4 * q:c16 * 16 + 4 * q + 4] = v[c16]
    err = (rec - full).abs().max().item()
    assert err <= 2.0 ** -22 * full.abs().max().item(), err
    assert torch.all(rec[co:] == 0) and torch.all(rec[:, ci:] == 0)
