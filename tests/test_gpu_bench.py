"""bench.py's BASELINE legs end to end on the GPU (short runs): CASIA with DACP + ECDA forced on
at SNR 0 / 10 dB (configs[3]) and the mixed-corpus K-fold sweep (configs[4])."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-data-path",
                        "--fp32-steps", "0"] + list(args), cwd=ROOT, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("snr", [0, 10])
def test_casia_forced_ecda_leg(snr):
    line = _bench("--flavor", "casia", "--force-ecda", "--snr", str(snr), "--steps", "6", "--warmup", "2")
    assert line["config"]["flavor"] == "casia" and line["config"]["snr_db"] == snr
    assert "configs[3]" in line["config"]["workload"]
    assert line["ecda_on_last_step"] == 1.0 and line["mask_sum_last_step"] > 1
    assert "scl_loss" in line["losses_last_step"] and line["losses_last_step"]["scl_loss"] == 0.0
    assert line["value"] > 0


def test_mixed_kfold_leg():
    line = _bench("--mixed", "--folds", "3", "--steps", "6", "--warmup", "3")
    assert line["config"]["flavor"] == "mixed"
    f = line["folds"]
    assert [x["fold"] for x in f] == [0, 1, 2]
    assert all(x["utterances"] == 6 * 64 and x["value"] > 0 for x in f)
    assert len({x["train_utterances"] for x in f}) > 1          # folds differ
    tot = sum(x["utterances"] for x in f) / sum(x["seconds"] for x in f)
    assert abs(line["value"] - tot) < 1e-6 * tot
    assert 2 * 64 * 100 <= f[0]["avg_valid_frames_per_step"] <= 2 * 64 * 300
