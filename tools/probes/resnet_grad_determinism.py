"""Run-to-run determinism of the ResNet GPU backward (two identical models, same batch): the
max relative difference of every weight gradient, with and without the split-K fold."""
import sys

import torch

sys.path.insert(0, ".")
from distributedtensorflowexample_amd.models.resnet import ResNet50, synthetic_imagenet  # noqa

dev = torch.device("cuda:0")
stages = [(64, 1, 1), (128, 1, 2)]
x, y = synthetic_imagenet(32, dev, size=112, seed=5, num_classes=10)
ms = [ResNet50(dev, seed=6, stages=stages, num_classes=10) for _ in range(3)]
ms[2].enable_splitk_fold()
gs = []
for m in ms:
    m.forward_backward(x, y)
    gs.append(m.materialize_grads().clone() if m._fold else m.params.grad.clone())
P = ms[0].params
worst = {}
for name, (off, shape) in P.offsets.items():
    n = 1
    for d in shape:
        n *= d
    a, b, c = gs[0][off:off + n], gs[1][off:off + n], gs[2][off:off + n]
    sc = a.abs().max().item() + 1e-30
    worst[name] = ((a - b).abs().max().item() / sc, (a - c).abs().max().item() / sc)
for name, (d01, d02) in sorted(worst.items(), key=lambda kv: -kv[1][0])[:12]:
    print("%-32s run-to-run %.3e   vs fold %.3e" % (name, d01, d02))
print("folded:", [n for n, v in ms[2]._planes.items() if v is not None])
