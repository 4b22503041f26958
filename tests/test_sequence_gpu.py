"""Ulysses SP module on the GPU (world 1: the all-to-alls are copies; the layout
transforms and the HIP attention kernels -- LDS kernel at S=128, flash at S=256 -- are
real), against the direct kernel call."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Solo:
    rank, world_size = 0, 1

    def all_to_all(self, out, inp):
        return out.copy_(inp)


@pytest.mark.parametrize("seq", [128, 256])
def test_ulysses_world1_matches_kernel(gpu, seq):
    from distributedtensorflowexample_amd.ops import transformer as T
    from distributedtensorflowexample_amd.parallel.sequence import ulysses_attention

    B, NH = 2, 12
    g = torch.Generator().manual_seed(5)
    qkv = (torch.randn(B * seq, 3 * NH * 64, generator=g) * 0.5).to(torch.bfloat16).to(gpu)
    dout = torch.randn(B * seq, NH * 64, generator=g).to(torch.bfloat16).to(gpu)
    kmask = torch.zeros(B, seq, device=gpu)
    kmask[1, seq - 7:] = -10000.0
    o_ref, lse = T.attn_fwd(qkv, B, seq, NH, kmask)
    d_ref = T.attn_bwd(qkv, o_ref, dout, lse, B, seq, NH, kmask)
    x = qkv.clone().requires_grad_(True)
    o = ulysses_attention(x, _Solo(), B, seq, NH, kmask)
    o.backward(dout)
    torch.cuda.synchronize()
    assert torch.equal(o, o_ref)
    assert (x.grad.float() - d_ref.float()).abs().max().item() < 1e-2
