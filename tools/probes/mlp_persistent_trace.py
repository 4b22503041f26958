"""Where a step of the persistent MLP engine spends its time: in-kernel s_memrealtime stamps
(100 MHz) per (workgroup, step), steady-state steps 8..63, medians in microseconds.

Stamps (csrc/kernels/mlp_persistent.hip): W1 blocks 0 before / 1 after the dz1 wait, 2 after
the barrier, 3 after the W1 update (Wt barrier), 4 after the slab stores; head waves 5 before /
6 after their wait, 7 after their stores; small blocks 0 / 1 around their wait, 2 published.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from distributedtensorflowexample_amd.data.synthetic import mnist_like_device  # noqa: E402
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.ops._ext import hip  # noqa: E402
from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer  # noqa: E402


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


def main():
    dev = torch.device("cuda:0")
    p = init_params(dev, seed=1234)
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(p, x, y, 100, 0.001)
    tr.run_persistent(100)
    nblk, ts = hip().mlp_persistent_blocks() + 100, hip().mlp_persistent_trace_steps()
    trace = torch.zeros(nblk, ts, 12, dtype=torch.int64, device=dev)
    tr.run_persistent(ts + 1, trace=trace)
    torch.cuda.synchronize()
    tr.check()
    T = trace.cpu().double() * 0.01  # ticks -> us
    nw1 = 98
    W, S = T[:nw1], T[nw1:nw1 + 7]
    hb = list(range(nw1 + 7, nw1 + 107))  # head blocks (row = block - 105)
    out = {}
    steps = range(8, ts - 1)
    out["period"] = med([W[:, t + 1, 3].median().item() - W[:, t, 3].median().item() for t in steps])
    out["w1_dz_wait"] = med([(W[:, t, 1] - W[:, t, 0]).median().item() for t in steps])
    out["w1_barrier1"] = med([(W[:, t, 2] - W[:, t, 1]).median().item() for t in steps])
    out["w1_update"] = med([(W[:, t, 3] - W[:, t, 2]).median().item() for t in steps])
    out["w1_phaseB"] = med([(W[:, t, 4] - W[:, t, 3]).median().item() for t in steps])
    H = T[hb]
    out["head_wait"] = med([(H[:, t, 6] - H[:, t, 5]).median().item() for t in steps])
    out["head_compute_store"] = med([(H[:, t, 7] - H[:, t, 6]).median().item() for t in steps])
    for w in range(3):
        out["head_wave%d_got_minus_wave3" % w] = med(
            [(H[:, t, 8 + w] - H[:, t, 6]).median().item() for t in steps])
    out["head_sync_to_stored"] = med([(H[:, t, 7] - H[:, t, 11]).median().item() for t in steps])
    out["head_wave3_got_to_sync"] = med([(H[:, t, 11] - H[:, t, 6]).median().item() for t in steps])
    # hand-offs: last producer done -> consumer sees data
    out["slab_last_store_to_head_got_med"] = med(
        [(H[:, t, 6] - W[:, t, 4].max()).median().item() for t in steps])
    out["slab_spread_first_last"] = med([(W[:, t, 4].max() - W[:, t, 4].min()).item() for t in steps])
    out["head_last_store_to_w1_got_med"] = med(
        [(W[:, t + 1, 1] - H[:, t, 7].max()).median().item() for t in steps])
    out["head_spread_first_last"] = med([(H[:, t, 7].max() - H[:, t, 7].min()).item() for t in steps])
    out["small_wait"] = med([(S[:, t, 1] - S[:, t, 0]).median().item() for t in steps])
    out["small_publish_to_head_got"] = med(
        [(H[:, t, 6] - S[:, t, 2].max()).median().item() for t in steps])
    print(json.dumps({k: round(v, 3) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
