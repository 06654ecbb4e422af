"""Helpers to replay the golden fixtures (tests/golden/*.npz) through a stepper."""
import glob
import json
import os

import numpy as np

from oracle import dad_oracle, synth

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TREE_FLAVOR = {"IEMOCAP": "iemocap", "CASIA": "casia", "EMODB": "emodb"}
# config keys the step reads (copied from the fixture's dump of the reference config module)
_KEYS = set(dad_oracle.FLAVOR_DEFAULTS["iemocap"])


def variants():
    # step fixtures (gen_golden.py); the data-path / eval-path fixtures data_*.npz, eval_*.npz
    # (gen_data_golden.py) are replayed by test_data_cpu.py, test_gpu_data.py, test_gpu_eval.py
    return sorted(n for n in (os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))
                  if not n.startswith(("data_", "eval_", "pretrain_")))


def load(name):
    d = dict(np.load(os.path.join(GOLDEN_DIR, name + ".npz")))
    spec = json.loads(str(d["variant_json"]))
    refcfg = json.loads(str(d["cfg_json"]))
    flavor = TREE_FLAVOR[spec["tree"]]
    cfg = dad_oracle.make_cfg(flavor, **{k: v for k, v in refcfg.items() if k in _KEYS})
    return d, spec, cfg


def schedule(d):
    """[(step_index, epoch)] in fixture order; each step starts from goldens.state()."""
    return [(s, int(d["s%d_epoch" % s])) for s in range(int(d["n_steps"]))]


def state(spec, step):
    return synth.make_state(spec["seed"], step, tau_range=tuple(spec.get("tau_range", (0.55, 0.9))))


def problem(spec):
    W1, b1, W2, b2, _ = synth.init_weights(spec["seed"])
    return W1, b1, W2, b2


def step_inputs(spec, step):
    return synth.make_step_inputs(spec["seed"], step, spec["B"], spec["T"], snr_db=spec.get("snr_db", 5.0))


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))
