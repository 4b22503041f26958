"""gflags-style command-line flags (the ``tf.app.flags`` API of main.py:26-39).

``DEFINE_string/integer/float/boolean`` register a flag; the global
:data:`FLAGS` parses ``sys.argv`` lazily on the first attribute access (the
reference calls ``main()`` directly, so TF parses on first ``FLAGS.x``, see
SURVEY §2.2 T11).  Accepted syntax: ``--name value``, ``--name=value``, and
for booleans ``--name`` / ``--noname``.  Unknown flags raise, like absl.

The reference's eight flags and defaults are declared by
:func:`define_reference_flags` (main.py:28-37); the framework adds
``--strategy``, ``--synthetic``, ``--dataset_size`` and friends.
"""
from __future__ import annotations

import sys


class FlagError(ValueError):
    pass


class _Flag:
    __slots__ = ("name", "default", "help", "parser", "value", "kind")

    def __init__(self, name, default, help_, parser, kind):
        self.name, self.default, self.help, self.parser, self.kind = name, default, help_, parser, kind
        self.value = default


def _parse_bool(s):
    v = str(s).strip().lower()
    if v in ("1", "true", "t", "yes", "y"):
        return True
    if v in ("0", "false", "f", "no", "n"):
        return False
    raise FlagError("not a boolean: %r" % s)


class FlagValues:
    def __init__(self):
        object.__setattr__(self, "_flags", {})
        object.__setattr__(self, "_parsed", False)
        object.__setattr__(self, "_argv", None)

    # -- definition -----------------------------------------------------------
    def _define(self, name, default, help_, parser, kind):
        if name in self._flags:
            raise FlagError("flag --%s defined twice" % name)
        self._flags[name] = _Flag(name, parser(default) if default is not None else None, help_,
                                  parser, kind)

    # -- parsing ------------------------------------------------------------
    def __call__(self, argv=None, known_only=False):
        """Parse ``argv`` (default sys.argv); returns the positional remainder."""
        argv = list(sys.argv if argv is None else argv)
        rest = [argv[0]] if argv else []
        i = 1
        while i < len(argv):
            a = argv[i]
            if a == "--":
                rest.extend(argv[i + 1:])
                break
            if not a.startswith("-") or a == "-":
                rest.append(a)
                i += 1
                continue
            body = a.lstrip("-")
            name, eq, val = body.partition("=")
            if name in ("help", "h", "helpfull") and name not in self._flags:
                print("flags:\n" + self.help())
                raise SystemExit(0)
            f = self._flags.get(name)
            if f is None and name.startswith("no") and name[2:] in self._flags \
                    and self._flags[name[2:]].kind == "bool" and not eq:
                self._flags[name[2:]].value = False
                i += 1
                continue
            if f is None:
                if known_only:
                    rest.append(a)
                    i += 1
                    continue
                raise FlagError("unknown command line flag %r" % a)
            if not eq:
                if f.kind == "bool" and (i + 1 >= len(argv) or argv[i + 1].startswith("-")
                                         or argv[i + 1].lower() not in
                                         ("true", "false", "1", "0", "t", "f", "yes", "no")):
                    f.value = True
                    i += 1
                    continue
                if i + 1 >= len(argv):
                    raise FlagError("flag --%s needs a value" % name)
                val = argv[i + 1]
                i += 1
            try:
                f.value = f.parser(val)
            except (TypeError, ValueError) as e:
                raise FlagError("bad value %r for --%s: %s" % (val, name, e))
            i += 1
        object.__setattr__(self, "_parsed", True)
        object.__setattr__(self, "_argv", rest)
        return rest

    def _ensure(self):
        if not self._parsed:
            self(sys.argv, known_only=True)

    def __getattr__(self, name):
        flags = object.__getattribute__(self, "_flags")
        if name not in flags:
            raise AttributeError(name)
        self._ensure()
        return flags[name].value

    def __setattr__(self, name, value):
        if name not in self._flags:
            raise AttributeError("no flag --%s" % name)
        self._flags[name].value = value

    def __contains__(self, name):
        return name in self._flags

    def flag_values_dict(self):
        self._ensure()
        return {k: f.value for k, f in self._flags.items()}

    def reset(self):
        """Back to defaults and unparsed (tests)."""
        for f in self._flags.values():
            f.value = f.default
        object.__setattr__(self, "_parsed", False)

    def help(self):
        return "\n".join("  --%s (default %r): %s" % (k, f.default, f.help)
                         for k, f in sorted(self._flags.items()))


FLAGS = FlagValues()


def DEFINE_string(name, default, help, flag_values=FLAGS):  # noqa: N802 - TF API
    flag_values._define(name, default, help, str, "str")


def DEFINE_integer(name, default, help, flag_values=FLAGS):  # noqa: N802
    flag_values._define(name, default, help, lambda v: int(float(v)) if isinstance(v, str) and
                        "e" in v.lower() else int(v), "int")


def DEFINE_float(name, default, help, flag_values=FLAGS):  # noqa: N802
    flag_values._define(name, default, help, float, "float")


def DEFINE_boolean(name, default, help, flag_values=FLAGS):  # noqa: N802
    flag_values._define(name, default, help, _parse_bool, "bool")


DEFINE_bool = DEFINE_boolean


def define_reference_flags(flag_values=FLAGS):
    """The flags of main.py:28-37 with their defaults, plus framework extensions."""
    fv = flag_values
    if "job_name" in fv:
        return fv
    DEFINE_string("job_name", "ps", "Either 'ps' or 'worker'", fv)
    DEFINE_integer("task_index", 0, "Index of task within the job", fv)
    DEFINE_integer("batch_size", 100, "Batch size", fv)
    DEFINE_float("learning_rate", 0.001, "Learning rate", fv)
    DEFINE_integer("training_steps", 10 ** 7, "Training steps (1step = 1batch update", fv)
    DEFINE_string("logdir", "./tmp/mnist/1", "Log directory", fv)
    DEFINE_integer("num_workers", 2, "Number of workers", fv)
    DEFINE_integer("num_gpus", 1, "Number of gpus, less than or equal to num_workers", fv)
    # --- framework extensions (not in the reference) ---
    DEFINE_integer("num_ps", 1, "Number of parameter-server tasks (variables round-robin)", fv)
    DEFINE_string("strategy", "ps_async",
                  "ps_async (reference semantics) or mirrored (sync all-reduce DP)", fv)
    DEFINE_string("data_dir", "", "MNIST IDX directory (default: the reference's MNIST_data)", fv)
    DEFINE_boolean("synthetic", False, "Use synthetic MNIST-shaped data", fv)
    DEFINE_integer("base_port", 12222, "First port of the localhost cluster (utils.py:12)", fv)
    DEFINE_string("device", "auto", "auto | cuda | cpu (worker compute device)", fv)
    DEFINE_integer("log_every", 100, "Print step/cost/speed every N global steps", fv)
    DEFINE_integer("eval_every", 10000, "Test accuracy every N global steps", fv)
    DEFINE_float("save_model_secs", 30.0, "Chief checkpoint interval (Supervisor)", fv)
    DEFINE_float("save_summaries_secs", 30.0, "Chief step-rate summary interval", fv)
    DEFINE_boolean("use_locking", False, "Serialize PS updates per variable", fv)
    DEFINE_boolean("ps_fused_rpc", True,
                   "Worker: push + global_step increment + the next step's pull in one "
                   "pipelined round trip per ps task (False: three round trips, as the "
                   "reference's three session runs)", fv)
    DEFINE_float("ps_timeout_secs", 0.0,
                 "Worker: a ps silent this long on a request counts as lost and the worker "
                 "exits non-zero (0: wait indefinitely; a dead ps is detected at once)", fv)
    DEFINE_string("ps_device", "cpu",
                  "cpu: variables on the TCP parameter server (the reference) | gpu: variables "
                  "in one GPU-resident store on the chief worker's GPU, IPC-mapped by every "
                  "worker (pull / apply / global_step over xGMI; async PS only)", fv)
    DEFINE_string("cpu_affinity", "numa",
                  "async PS: numa = the ps tasks on GPU 0's NUMA node (--numa_node overrides), "
                  "8 cores each; worker i on 2 cores of its OWN GPU's node, after the ps tasks' "
                  "core positions; a slot that does not fit on its node is left unpinned "
                  "(warning) -- Hogwild applies and pulls of several connection threads "
                  "scattered over two sockets bounce the same cache lines across the socket "
                  "link | none", fv)
    DEFINE_integer("numa_node", -1, "--cpu_affinity numa: the ps process's node (-1: auto)", fv)
    DEFINE_integer("seed", 0, "Parameter init seed", fv)
    DEFINE_string("model", "mlp", "mlp (the reference) | bert | resnet50 (north-star configs); "
                  "async PS: mlp | softmax (softmax regression)", fv)
    DEFINE_string("hidden_units", "", "async PS, --model mlp: hidden layer widths, e.g. 256,128 "
                  "(default: the reference's 100)", fv)
    DEFINE_string("activation", "sigmoid", "async PS, --model mlp: hidden activation "
                  "(sigmoid | relu)", fv)
    DEFINE_string("model_config", "base", "base | tiny (tiny = CPU-sized variant of bert/resnet50)",
                  fv)
    DEFINE_integer("seq_len", 128, "BERT sequence length", fv)
    DEFINE_integer("image_size", 224, "ResNet input resolution", fv)
    DEFINE_string("dtype", "auto", "auto: fp32 for the MLP (reference dtype), bf16 for bert/resnet50",
                  fv)
    DEFINE_float("bucket_mb", 32.0, "All-reduce bucket size for generic DDP models (MiB)", fv)
    DEFINE_boolean("sync_replicas", False,
                   "ps_async strategy: aggregate each step's gradients over "
                   "--replicas_to_aggregate workers on the ps before ONE apply "
                   "(tf.train.SyncReplicasOptimizer); stale gradients are dropped", fv)
    DEFINE_integer("replicas_to_aggregate", 0,
                   "--sync_replicas: gradients averaged per step (0 = --num_workers; fewer "
                   "than --num_workers makes the slowest workers backups)", fv)
    DEFINE_boolean("zero1", False, "Autograd sync-DP path: shard the optimizer update over the "
                   "replicas (ZeRO-1: reduce-scatter, owner update, all-gather)", fv)
    DEFINE_float("dist_timeout_secs", 300.0,
                 "Sync DP: timeout of the gloo control-plane collectives (torch's default is "
                 "30 min); a rank whose peer died raises after at most this long", fv)
    DEFINE_float("peer_timeout_secs", 60.0,
                 "Sync DP fail-fast watchdog: a peer whose store heartbeat stalls this long is "
                 "lost -- RCCL is aborted and the rank exits with code 75 (0 = off)", fv)
    DEFINE_integer("check_replicas_every", 0,
                   "Sync DP debug check (SURVEY 5.2): every N steps compare every replica's "
                   "parameters with rank 0's and stop if they are not bit-identical (0 = off)", fv)
    return fv
