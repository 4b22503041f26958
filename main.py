"""Distributed training entry point -- the reference's ``main.py`` CLI, MI355X-native.

Same flags and defaults as the reference (main.py:28-37), same role dispatch:

    python main.py --job_name ps --task_index 0 --num_workers 2 --num_gpus 1
    python main.py --job_name worker --task_index 0 --num_workers 2 --num_gpus 1

``--strategy ps_async`` (default) reproduces the reference's asynchronous
parameter-server SGD (native C++ PS over TCP, fused HIP kernels on the
workers).  ``--strategy mirrored`` runs synchronous data parallelism, one
process per GPU (RANK/WORLD_SIZE/LOCAL_RANK from the launcher), gradients
all-reduced over RCCL/xGMI.  Launch whole clusters with
``python -m distributedtensorflowexample_amd.launch`` (replaces tmux) or the
``run_single_gpu.sh`` / ``run_multi_gpu.sh`` wrappers.
"""
from __future__ import annotations

import os
import signal
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from distributedtensorflowexample_amd import flags as flags_mod  # noqa: E402

flags_mod.define_reference_flags()
FLAGS = flags_mod.FLAGS


def _install_signal_handlers():
    """main.py:51-55: SIGHUP/SIGINT/SIGTERM -> exit(128 + signum)."""
    def shutdown(signum, frame):
        sys.exit(128 + signum)

    for s in (signal.SIGHUP, signal.SIGINT, signal.SIGTERM):
        signal.signal(s, shutdown)


def main(argv=None):
    FLAGS(sys.argv if argv is None else argv)
    from distributedtensorflowexample_amd.cluster import ClusterSpec, Server, cluster_spec
    from distributedtensorflowexample_amd.config import ConfigProto, GPUOptions, memory_fraction
    from distributedtensorflowexample_amd.data.mnist import read_data_sets

    _install_signal_handlers()

    if FLAGS.strategy == "mirrored" and FLAGS.model != "mlp":
        from distributedtensorflowexample_amd.train.mirrored_mlp import shutdown_mirrored
        from distributedtensorflowexample_amd.train.mirrored_models import train_model_mirrored

        train_model_mirrored(FLAGS)
        shutdown_mirrored()
        return 0
    if FLAGS.strategy == "mirrored":
        from distributedtensorflowexample_amd.train.mirrored_mlp import (shutdown_mirrored,
                                                                         train_mirrored)

        mnist = read_data_sets(FLAGS.data_dir or None, one_hot=True, seed=FLAGS.seed)
        train_mirrored(FLAGS, mnist)
        shutdown_mirrored()
        return 0
    if FLAGS.strategy != "ps_async":
        raise SystemExit("unknown --strategy %r" % FLAGS.strategy)

    # Cluster specification (main.py:46-48; num_ps is a flag here, 1 by default)
    spec = cluster_spec(FLAGS.num_workers, FLAGS.num_ps, base_port=FLAGS.base_port)
    cluster = ClusterSpec(spec)

    # GPU memory fraction (main.py:57-64)
    fraction = memory_fraction(FLAGS.num_workers, FLAGS.num_gpus)
    print("-" * 100)
    print("Per-process GPU memory fraction: {}".format(fraction))
    print("-" * 100, flush=True)
    gpu_options = GPUOptions(per_process_gpu_memory_fraction=fraction)

    if FLAGS.job_name == "ps":
        if getattr(FLAGS, "cpu_affinity", "none") == "numa":
            from distributedtensorflowexample_amd.config import (first_gpu_numa_node_sysfs,
                                                                 pin_to_numa_node, ps_cpu_slot)

            node = FLAGS.numa_node if FLAGS.numa_node >= 0 else first_gpu_numa_node_sysfs()
            pin_to_numa_node(0 if node is None else node, *ps_cpu_slot(FLAGS.task_index))
        # Quirk decided: the ps does not load MNIST; it serves
        # until a client asks it to shut down (or it is signalled).
        server = Server(cluster, job_name="ps", task_index=FLAGS.task_index)
        server.join()
    elif FLAGS.job_name == "worker":
        from distributedtensorflowexample_amd.config import apply_hip_schedule
        from distributedtensorflowexample_amd.train.worker import Worker

        # pinned first: the affinity of the calling thread is inherited by the threads started
        # after it, so the HIP runtime's threads (apply_hip_schedule may start them) follow
        if getattr(FLAGS, "cpu_affinity", "none") == "numa":
            from distributedtensorflowexample_amd.config import (first_gpu_numa_node_sysfs,
                                                                 pin_to_numa_node,
                                                                 worker_cpu_slot)

            from distributedtensorflowexample_amd.config import visible_gpu_index

            # the node of this worker's GPU (the launcher's HIP_VISIBLE_DEVICES)
            node = (FLAGS.numa_node if FLAGS.numa_node >= 0
                    else first_gpu_numa_node_sysfs(index=visible_gpu_index()))
            pin_to_numa_node(0 if node is None else node,
                             *worker_cpu_slot(FLAGS.task_index, FLAGS.num_ps))
        apply_hip_schedule()  # DTFX_HIP_SCHED (before the first GPU call)
        mnist = read_data_sets(FLAGS.data_dir or None, one_hot=True)
        config = ConfigProto(gpu_options=gpu_options)
        server = Server(cluster, job_name="worker", task_index=FLAGS.task_index, config=config)
        worker = Worker(FLAGS.job_name, FLAGS.task_index, server, FLAGS, device=FLAGS.device)
        worker.learn(mnist)
    else:
        raise SystemExit("--job_name must be 'ps' or 'worker'")
    return 0


if __name__ == "__main__":
    sys.exit(main())
