"""The data-parallel shape of the BERT-base / ResNet-50 steps on ONE GPU.

A world-W trainer runs rank 0's step with ``parallel.xgmi.SimulatedPeersComm``: the real
bucket hooks on the comm stream, the real bandwidth-mode two-shot all-reduce kernel per bucket
(its stores into W-1 "peer" slots, owner sum, gathers -- local HBM, flags pre-raised), and
every world > 1 default of the trainer (BERT: weight gradients on a side stream, no split-K
fold).  Against the 1-GPU step, each switch A/B'd in the same process, interleaved rounds:

  1gpu          comm None (the bench's step)
  dp            world W, trainer defaults, the bw kernel on 128 workgroups (pick_large_allreduce's
                default since round 5); BERT: the owner-sharded AdamW (reduce-scatter / shard
                AdamW / all-gather halves of the bw kernel) since round 6
  dp_rep        BERT: the replicated AdamW over all-reduced buckets (DTFX_BERT_ZERO1=0)
  dp_null       world W, all-reduce a no-op (the DP-mode trainer changes alone)
  dp_bw256 / 64 the bw kernel on all 256 / on 64 workgroups
  dp_prio_hi    the comm stream at the highest HIP stream priority (default: the lowest,
                the compute stream's)
  BERT: dp_nows (no weight-gradient stream), 1gpu_nofold (the 1-GPU step without the fold)
  ResNet: dp_ws (weight gradients on a side stream), dp_zero1 (the owner-sharded momentum SGD:
          reduce-scatter per bucket, SGD on the rank's shard, shards all-gathered beside the
          next forward -- DTFX_RESNET_ZERO1=1)

What this cannot show is link time: the all-reduce's bytes cross local HBM, not xGMI.

    python tools/probes/dp_sim.py --model bert [--world 8 --steps 10 --rounds 3]
"""
import argparse
import gc
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.parallel.xgmi import SimulatedPeersComm  # noqa: E402


class NullComm:
    """World-W communicator whose all-reduce does nothing (isolates the trainer's DP-mode
    changes from the comm kernels)."""

    def __init__(self, world):
        self.rank, self.world_size = 0, world

    def allreduce_sum_(self, t):
        return t

    def reduce_scatter(self, out, inp):
        return out

    def all_gather(self, out, inp):
        return out

    def broadcast_(self, t, root=0):
        return t


def make(model, variant, world, dev, a):
    env = {}
    if variant == "dp_nows":
        env["DTFX_BERT_WSTREAM"] = "0"
    if variant == "dp_rep":  # BERT: replicated AdamW over all-reduced buckets (rounds 4-5)
        env["DTFX_BERT_ZERO1"] = "0"
    if variant == "1gpu_nofold":
        env["DTFX_BERT_FOLD"] = "0"
    if variant == "dp_ws":
        env["DTFX_RESNET_WSTREAM"] = "1"
    if variant == "dp_zero1":
        env["DTFX_RESNET_ZERO1"] = "1"
    if variant == "dp_prio_hi":
        env["DTFX_COMM_PRIORITY"] = str(torch.cuda.Stream.priority_range()[1])
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        comm = None
        if variant.startswith("dp"):
            if variant == "dp_null":
                comm = NullComm(world)
            else:
                blocks = {"dp_bw256": 256, "dp_bw64": 64}.get(variant, 128)
                comm = SimulatedPeersComm(world, (24 << 20) if model == "bert" else (8 << 20),
                                          device=dev, bw_blocks=blocks)
        if model == "bert":
            from distributedtensorflowexample_amd.models.bert import BertConfig
            from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

            return BertTrainer(BertConfig.base(), a.batch or 128, 128, dev, comm=comm, data_seed=17)
        from distributedtensorflowexample_amd.train.resnet_trainer import ResNetTrainer

        return ResNetTrainer(a.batch or 256, dev, comm=comm)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["bert", "resnet50"], default="bert")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    if a.variants:
        variants = a.variants.split(",")
    elif a.model == "bert":
        variants = ["1gpu", "dp", "dp_null", "dp_nows", "dp_bw256", "dp_bw64", "dp_prio_hi",
                    "1gpu_nofold"]
    else:
        variants = ["1gpu", "dp", "dp_zero1", "dp_null", "dp_bw256", "dp_bw64", "dp_prio_hi", "dp_ws"]
    trainers = {}
    for v in variants:
        tr = make(a.model, v, a.world, dev, a)
        tr.run(3, True)  # eager warm step + capture + replay
        torch.cuda.synchronize()
        trainers[v] = tr
        print("[dp_sim] ready: %s" % v, file=sys.stderr, flush=True)
    res = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            tr = trainers[v]
            tr.run(2, True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.run(a.steps, True)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) * 1e3 / a.steps)
        print("[dp_sim] round done", file=sys.stderr, flush=True)
    base = sorted(res["1gpu"])[len(res["1gpu"]) // 2] if "1gpu" in res else None
    out = {"model": a.model, "world": a.world, "steps": a.steps, "rounds": a.rounds,
           "note": "rank 0 of a simulated world-%d job on one GPU: real bucket hooks, comm "
                   "stream and bw all-reduce kernels over local HBM (no xGMI link time)" % a.world,
           "ms_per_step": {}}
    for v in variants:
        med = sorted(res[v])[len(res[v]) // 2]
        out["ms_per_step"][v] = {"median": round(med, 3), "all": [round(t, 3) for t in res[v]],
                                 "vs_1gpu_pct": round(100 * (med / base - 1), 2) if base else None}
        try:
            loss, _ = trainers[v].stats()
            out["ms_per_step"][v]["final_loss"] = round(loss, 4)
        except Exception:  # noqa: BLE001
            pass
    print(json.dumps(out, indent=1), flush=True)
    trainers.clear()
    gc.collect()


if __name__ == "__main__":
    main()
