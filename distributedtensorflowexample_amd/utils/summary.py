"""TensorBoard summaries (``tf.summary.scalar`` / ``merge_all`` / ``FileWriter``).

The reference logs ``loss`` and ``accuracy`` every step to
``logdir + '_%d' % task_index`` (worker.py:92-96, 139).  :class:`FileWriter`
wraps the native C++ event writer (TFRecord framing + masked CRC32C, async
flush thread, ``csrc/host/event_writer.cpp``), so the files are readable by
TensorBoard.  Summaries are serialized ``tensorflow.Summary`` protos; since
``Summary.value`` is a repeated field, concatenating serialized summaries is
exactly ``merge``.
"""
from __future__ import annotations

import os

from ..ops import host


def scalar(tag, value):
    """Serialized Summary with one simple_value (tf.summary.scalar)."""
    return host().summary_scalars({str(tag): float(value)})


def merge(summaries):
    """tf.summary.merge: concatenation of serialized Summary protos."""
    return b"".join(bytes(s) for s in summaries)


class FileWriter:
    def __init__(self, logdir, graph=None, max_queue=10, flush_secs=120, filename_suffix=""):
        os.makedirs(logdir, exist_ok=True)
        self._logdir = logdir
        self._w = host().EventWriter(logdir, float(flush_secs), filename_suffix)

    def get_logdir(self):
        return self._logdir

    @property
    def path(self):
        return self._w.path

    def add_summary(self, summary, global_step=None):
        """``summary``: serialized Summary bytes or a {tag: float} dict."""
        step = int(global_step or 0)
        if isinstance(summary, dict):
            self._w.add_scalars({str(k): float(v) for k, v in summary.items()}, step)
        else:
            self._w.add_summary(bytes(summary), step)

    def add_graph(self, graph_def):
        """``FileWriter.add_graph``: one Event carrying the serialized GraphDef (bytes, or a
        ``utils.graph.GraphDefBuilder``), shown by TensorBoard's Graphs tab."""
        from .graph import graph_event

        if hasattr(graph_def, "to_bytes"):
            graph_def = graph_def.to_bytes()
        self._w.add_event(graph_event(bytes(graph_def)))

    def add_scalars(self, values, global_step):
        self._w.add_scalars({str(k): float(v) for k, v in values.items()}, int(global_step))

    def add_scalar_series(self, tags, steps, values):
        """Bulk path: one event per step from a [n, len(tags)] array."""
        self._w.add_scalar_series(list(tags), [int(s) for s in steps],
                                  [[float(v) for v in row] for row in values])

    def flush(self):
        self._w.flush()

    def close(self):
        self._w.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_events(path):
    """[{'step', 'wall_time', 'scalars': {...}, 'graph_def'?: bytes}] of an event file
    (tests/tools)."""
    h = host()
    return [h.parse_event(r) for r in h.read_records(path)]
