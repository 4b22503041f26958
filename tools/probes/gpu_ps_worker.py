"""One async-PS worker (chief) training through the GPU-resident parameter store in-process
(ps task started in the same process) -- for rocprofv3 kernel traces of the device-side
pull / apply / global_step ops.  Prints global steps/sec."""
import os
import socket
import sys
import tempfile
import time
import types

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from distributedtensorflowexample_amd.cluster import Server  # noqa: E402
from distributedtensorflowexample_amd.data.mnist import read_data_sets  # noqa: E402
from distributedtensorflowexample_amd.train.worker import Worker  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    spec = {"ps": ["127.0.0.1:%d" % port], "worker": ["127.0.0.1:1"]}
    ps = Server(spec, "ps", 0)
    try:
        fl = types.SimpleNamespace(batch_size=100, learning_rate=0.001, training_steps=steps,
                                   logdir=os.path.join(tempfile.mkdtemp(), "m"), log_every=10 ** 9,
                                   eval_every=10 ** 9, save_model_secs=1e9,
                                   save_summaries_secs=1e9, use_locking=False, seed=0,
                                   device="cuda", ps_device="gpu", num_workers=1)
        w = Worker("worker", 0, Server(spec, "worker", 0), fl, device="cuda", log=print)
        data = read_data_sets(seed=0)
        t0 = time.time()
        h = w.learn(data)
        dt = time.time() - t0
        print("steps %d  %.1f global steps/s  loss %.4f -> %.4f" % (len(h), len(h) / dt, h[0][1],
                                                                  h[-1][1]))
    finally:
        ps.stop()


if __name__ == "__main__":
    main()
