"""The training graph as a ``tensorflow.GraphDef`` -- what TF's Supervisor writes for the chief.

The reference builds a TF graph (worker.py:8-103) and its chief Supervisor writes it to the
log directory at session start (worker.py:107-118; TF: ``graph.pbtxt`` in ``logdir`` and a
``graph_def`` event through the summary writer), which is what TensorBoard's Graphs tab shows.
This framework runs no dataflow graph -- the step is hand-written HIP kernels -- so the GraphDef
is *described*: :func:`reference_mlp_graph` lays out the reference's ops (the global replica
and ``global_step`` on the ps, the local replica + forward / loss / gradient / remote apply /
sync / accuracy / summary ops on the worker) with the variable names and shapes taken from the
variable registry (``variables.py``), and :class:`GraphDefBuilder` encodes it as the GraphDef
protobuf (binary, for the event file) and protobuf text format (``graph.pbtxt``).

Encoding (tensorflow/core/framework/graph.proto, node_def.proto, attr_value.proto):
GraphDef {1: repeated NodeDef node, 4: VersionDef versions {1: producer}};
NodeDef {1: name, 2: op, 3: repeated input, 4: device, 5: map<string, AttrValue> attr};
AttrValue {6: DataType type, 7: TensorShapeProto shape {2: repeated Dim {1: size}}, 2: s}.
"""
from __future__ import annotations

import struct
import time

DT = {"float32": (1, "DT_FLOAT"), "int32": (3, "DT_INT32"), "int64": (9, "DT_INT64"),
      "string": (7, "DT_STRING"), "bool": (10, "DT_BOOL")}
PRODUCER = 27  # TF 1.x-era GraphDef producer version


def _varint(n):
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wire):
    return _varint((field << 3) | wire)


def _bytes_field(field, data):
    if isinstance(data, str):
        data = data.encode()
    return _key(field, 2) + _varint(len(data)) + data


def _varint_field(field, v):
    return _key(field, 0) + _varint(v)


def _attr_value(v):
    """AttrValue from ('type', dtype) | ('shape', dims) | ('s', str)."""
    kind, val = v
    if kind == "type":
        return _varint_field(6, DT[val][0])
    if kind == "shape":
        shp = b"".join(_bytes_field(2, _varint_field(1, d if d >= 0 else (1 << 64) + d))
                       for d in val)
        return _bytes_field(7, shp)
    if kind == "s":
        return _bytes_field(2, val)
    raise ValueError("unsupported attr kind %r" % kind)


def _attr_text(v):
    kind, val = v
    if kind == "type":
        return "type: %s" % DT[val][1]
    if kind == "shape":
        return "shape { %s }" % " ".join("dim { size: %d }" % d for d in val) if val else \
            "shape { }"
    return 's: "%s"' % val


class GraphDefBuilder:
    def __init__(self):
        self.nodes = []

    def node(self, name, op, inputs=(), device="", **attrs):
        self.nodes.append((name, op, list(inputs), device, attrs))
        return name

    def to_bytes(self):
        out = bytearray()
        for name, op, inputs, device, attrs in self.nodes:
            nd = _bytes_field(1, name) + _bytes_field(2, op)
            for i in inputs:
                nd += _bytes_field(3, i)
            if device:
                nd += _bytes_field(4, device)
            for k in sorted(attrs):
                nd += _bytes_field(5, _bytes_field(1, k) + _bytes_field(2, _attr_value(attrs[k])))
            out += _bytes_field(1, nd)
        out += _bytes_field(4, _varint_field(1, PRODUCER))
        return bytes(out)

    def to_pbtxt(self):
        lines = []
        for name, op, inputs, device, attrs in self.nodes:
            lines.append("node {")
            lines.append('  name: "%s"' % name)
            lines.append('  op: "%s"' % op)
            lines += ['  input: "%s"' % i for i in inputs]
            if device:
                lines.append('  device: "%s"' % device)
            for k in sorted(attrs):
                lines.append("  attr {")
                lines.append('    key: "%s"' % k)
                lines.append("    value {")
                lines.append("      " + _attr_text(attrs[k]))
                lines.append("    }")
                lines.append("  }")
            lines.append("}")
        lines.append("versions {")
        lines.append("  producer: %d" % PRODUCER)
        lines.append("}")
        return "\n".join(lines) + "\n"


def graph_event(graph_def, wall_time=None):
    """Serialized ``tensorflow.Event`` carrying a graph: {1: wall_time, 4: graph_def}."""
    w = time.time() if wall_time is None else float(wall_time)
    return _key(1, 1) + struct.pack("<d", w) + _bytes_field(4, graph_def)


def reference_mlp_graph(global_vars, trainable, task_index=0, batch_size=-1,
                        learning_rate=0.001):
    """The reference worker's graph (worker.py:8-103) over the registry's variables.

    ``global_vars``: ``get_vars('global', False)`` (ps variables incl. global_step);
    ``trainable``: ``get_vars('global')`` (the four dense kernels / biases, creation order)."""
    g = GraphDefBuilder()
    ps = "/job:ps/task:0"
    wdev = "/job:worker/task:%d/gpu:0" % task_index
    gscope = trainable[0].name.split("/")[0] if trainable else "global"
    for v in global_vars:
        dt = "float32" if v.dtype == "float32" else "int32"
        g.node(v.name, "VariableV2", device=ps, dtype=("type", dt), shape=("shape", list(v.shape)))
    step = next((v.name for v in global_vars if v.name.endswith("global_step")), None)
    if step:
        one = g.node(gscope + "/Const", "Const", device=ps, dtype=("type", "int32"))
        g.node(gscope + "/AssignAdd", "AssignAdd", [step, one], device=ps)  # counter_op
    # local replica (worker.py:34-40): the same layer names under "local"
    local = {}
    for v in trainable:
        ln = "local/" + v.name.split("/", 1)[1]
        local[v.name] = g.node(ln, "VariableV2", device=wdev, dtype=("type", "float32"),
                               shape=("shape", list(v.shape)))
    x = g.node("local/Placeholder", "Placeholder", device=wdev, dtype=("type", "float32"),
               shape=("shape", [batch_size, trainable[0].shape[0]]))
    y = g.node("local/Placeholder_1", "Placeholder", device=wdev, dtype=("type", "float32"),
               shape=("shape", [batch_size, trainable[-1].shape[-1]]))
    names = [local[v.name] for v in trainable]
    h = x
    nl = len(names) // 2
    for li in range(nl):
        k, b = names[2 * li], names[2 * li + 1]
        pre = k.rsplit("/", 1)[0]
        mm = g.node(pre + "/MatMul", "MatMul", [h, k], device=wdev, T=("type", "float32"))
        h = g.node(pre + "/BiasAdd", "BiasAdd", [mm, b], device=wdev, T=("type", "float32"))
        if li < nl - 1:
            h = g.node(pre + "/Sigmoid", "Sigmoid", [h], device=wdev, T=("type", "float32"))
    logits = h
    net = g.node("local/Softmax", "Softmax", [logits], device=wdev)
    xent = g.node("local/SoftmaxCrossEntropyWithLogits", "SoftmaxCrossEntropyWithLogits",
                  [logits, y], device=wdev)
    loss = g.node("local/Mean", "Mean", [xent], device=wdev)
    # compute_gradients on the local replica, apply_gradients to the GLOBAL variables
    # (worker.py:70-79): one ApplyGradientDescent per (global var, local grad) pair, on the ps
    lr = g.node("local/GradientDescent/learning_rate", "Const", device=wdev,
                dtype=("type", "float32"))
    grads = g.node("local/gradients/Fill", "Fill", [loss], device=wdev)
    upd = []
    for v in trainable:
        gn = g.node("local/gradients/%s_grad" % local[v.name].split("/", 1)[1].replace("/", "_"),
                    "Identity", [grads], device=wdev)
        upd.append(g.node("local/GradientDescent/update_%s/ApplyGradientDescent" % v.name,
                          "ApplyGradientDescent", [v.name, lr, gn], device=ps))
    g.node("local/GradientDescent", "NoOp", ["^" + u for u in upd], device=wdev)
    # sync_op (worker.py:81-85): local <- global
    asg = [g.node("local/Assign%s" % ("" if i == 0 else "_%d" % i), "Assign",
                  [local[v.name], v.name], device=wdev) for i, v in enumerate(trainable)]
    g.node("local/group_deps", "NoOp", ["^" + a for a in asg], device=wdev)
    # accuracy + summaries (worker.py:87-96)
    am = g.node("local/ArgMax", "ArgMax", [net], device=wdev)
    am1 = g.node("local/ArgMax_1", "ArgMax", [y], device=wdev)
    eq = g.node("local/Equal", "Equal", [am, am1], device=wdev)
    cast = g.node("local/Cast", "Cast", [eq], device=wdev)
    acc = g.node("local/Mean_1", "Mean", [cast], device=wdev)
    s1 = g.node("local/loss", "ScalarSummary", [loss], device="/job:worker/task:%d/cpu:0"
                % task_index)
    s2 = g.node("local/accuracy", "ScalarSummary", [acc], device="/job:worker/task:%d/cpu:0"
                % task_index)
    g.node("Merge/MergeSummary", "MergeSummary", [s1, s2],
           device="/job:worker/task:%d/cpu:0" % task_index)
    return g
