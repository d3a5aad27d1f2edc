"""The framework's HSA runtime defaults (distributed_neural_network_amd/hsa_env.py): applied at
package import, an explicit environment value wins, DNN_HSA_DEFAULTS=0 applies none."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = "import distributed_neural_network_amd, os; print(os.environ.get('HSA_ALLOCATE_QUEUE_DEV_MEM'))"


def _probe(**env):
    e = {k: v for k, v in os.environ.items() if k not in ("HSA_ALLOCATE_QUEUE_DEV_MEM", "DNN_HSA_DEFAULTS")}
    e.update(env)
    e["PYTHONPATH"] = ROOT
    return subprocess.run([sys.executable, "-c", PROBE], env=e, capture_output=True, text=True, check=True).stdout.strip()


def test_defaults_apply_at_import():
    assert _probe() == "1"


def test_explicit_value_wins():
    assert _probe(HSA_ALLOCATE_QUEUE_DEV_MEM="0") == "0"


def test_opt_out():
    assert _probe(DNN_HSA_DEFAULTS="0") == "None"


def test_ranks_of_a_multi_rank_job_keep_the_runtime_defaults():
    assert _probe(WORLD_SIZE="8") == "None"
    assert _probe(WORLD_SIZE="1") == "1"


def test_strip_removes_only_what_apply_set():
    from distributed_neural_network_amd import hsa_env

    env = {"HSA_ALLOCATE_QUEUE_DEV_MEM": "1", "DNN_HSA_DEFAULTED": "HSA_ALLOCATE_QUEUE_DEV_MEM", "X": "y"}
    assert hsa_env.strip(env) == {"X": "y"}
    user = {"HSA_ALLOCATE_QUEUE_DEV_MEM": "1", "X": "y"}  # set by the user: kept
    assert hsa_env.strip(dict(user)) == user
