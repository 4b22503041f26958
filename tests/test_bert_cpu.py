"""Tiny BERT MLM step on the CPU reference paths vs a torch-autograd model."""
import math

import torch

from distributedtensorflowexample_amd.models.bert import BertConfig, BertMLM, synthetic_mlm_batch


def _ref_loss(P, cfg, ids, tt, pos, labels, n_valid):
    F = torch.nn.functional
    B, S = ids.shape
    H, nh = cfg.hidden, cfg.heads
    x = P["embeddings/word_embeddings"][ids.long()] + P["embeddings/position_embeddings"][:S] + \
        P["embeddings/token_type_embeddings"][tt.long()]
    h = F.layer_norm(x, (H,), P["embeddings/LayerNorm/gamma"], P["embeddings/LayerNorm/beta"], cfg.eps)
    for l in range(cfg.layers):
        p = "encoder/layer_%d/" % l
        qkv = h @ P[p + "attention/qkv/kernel"].t() + P[p + "attention/qkv/bias"]
        q, k, v = qkv.view(B, S, 3, nh, 64).permute(2, 0, 3, 1, 4)
        a = torch.softmax(q @ k.transpose(-1, -2) / 8, -1) @ v
        a = a.permute(0, 2, 1, 3).reshape(B, S, H)
        a = a @ P[p + "attention/output/dense/kernel"].t() + P[p + "attention/output/dense/bias"] + h
        h1 = F.layer_norm(a, (H,), P[p + "attention/output/LayerNorm/gamma"],
                          P[p + "attention/output/LayerNorm/beta"], cfg.eps)
        g = F.gelu(h1 @ P[p + "intermediate/dense/kernel"].t() + P[p + "intermediate/dense/bias"],
                   approximate="tanh")
        f = g @ P[p + "output/dense/kernel"].t() + P[p + "output/dense/bias"] + h1
        h = F.layer_norm(f, (H,), P[p + "output/LayerNorm/gamma"], P[p + "output/LayerNorm/beta"],
                         cfg.eps)
    hm = h.reshape(B * S, H)[pos]
    t = F.gelu(hm @ P["cls/predictions/transform/dense/kernel"].t() +
               P["cls/predictions/transform/dense/bias"], approximate="tanh")
    t = F.layer_norm(t, (H,), P["cls/predictions/transform/LayerNorm/gamma"],
                     P["cls/predictions/transform/LayerNorm/beta"], cfg.eps)
    logits = t @ P["embeddings/word_embeddings"][:cfg.vocab_size].t() + \
        P["cls/predictions/output_bias"][:cfg.vocab_size]
    return F.cross_entropy(logits, labels.long(), ignore_index=-100, reduction="sum") / n_valid


def test_bert_tiny_step_matches_autograd():
    torch.manual_seed(0)
    cfg = BertConfig.tiny()
    m = BertMLM(cfg, "cpu", seed=3)
    ids, tt, pos, lab, nv = synthetic_mlm_batch(cfg, 2, 32, "cpu", seed=1, pad_to=16)
    assert lab.numel() % 16 == 0 and nv == 2 * round(0.15 * 32)
    loss, acc = m.forward_backward(ids, tt, pos, lab, n_valid=nv)
    P = {k: v.clone().requires_grad_(True) for k, v in m.params.state_dict().items()}
    ref = _ref_loss(P, cfg, ids, tt, pos, lab, nv)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 0.02 * ref.item()
    assert math.isfinite(acc.item())
    for name in ["encoder/layer_0/attention/qkv/kernel", "encoder/layer_1/output/dense/kernel",
                 "embeddings/word_embeddings", "cls/predictions/transform/dense/kernel",
                 "embeddings/LayerNorm/gamma", "encoder/layer_0/intermediate/dense/bias"]:
        g, r = m.params.G(name).flatten(), P[name].grad.flatten()
        cos = torch.dot(g, r) / (g.norm() * r.norm() + 1e-30)
        assert cos > 0.98, (name, cos.item())
        assert abs(g.norm() / r.norm() - 1) < 0.1, (name, (g.norm() / r.norm()).item())


def test_bert_tiny_adam_decreases_loss():
    cfg = BertConfig.tiny()
    m = BertMLM(cfg, "cpu", seed=0)
    batch = synthetic_mlm_batch(cfg, 2, 32, "cpu", seed=5, pad_to=16)
    losses = []
    for step in range(1, 6):
        loss, _ = m.forward_backward(*batch[:4], n_valid=batch[4])
        m.adam_step(1e-3, step)
        losses.append(loss.item())
    assert losses[-1] < losses[0]


def test_bert_base_param_count_and_buckets():
    cfg = BertConfig.base()
    from distributedtensorflowexample_amd.models.bert import param_layout

    n = sum(math.prod(s) for _, s, _ in param_layout(cfg))
    assert 109e6 < n < 111e6   # BERT-base with a 64-padded vocabulary
