"""Static checks of the launch scripts and repo contracts (reference: test_run_sh.py)."""
import json
import os
import stat

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["run.sh", "run-in-vm.sh"])
def test_script_exists_executable_with_shebang(name):
    path = os.path.join(ROOT, name)
    assert os.path.isfile(path)
    assert os.stat(path).st_mode & stat.S_IXUSR
    with open(path) as f:
        first = f.readline()
    assert first.startswith("#!") and "bash" in first


@pytest.mark.parametrize("name", ["run.sh", "run-in-vm.sh"])
def test_script_builds_kernels_and_starts_api(name):
    text = open(os.path.join(ROOT, name)).read()
    assert "setup.py build_ext" in text
    assert "main.py" in text
    assert "set -euo pipefail" in text


def test_vm_script_listens_on_all_interfaces():
    assert "0.0.0.0" in open(os.path.join(ROOT, "run-in-vm.sh")).read()


def test_scripts_do_not_force_cpu_wheels():
    for name in ("run.sh", "run-in-vm.sh"):
        text = open(os.path.join(ROOT, name)).read()
        assert "download.pytorch.org/whl/cpu" not in text and "pip install" not in text


def test_log_config_is_valid_dictconfig():
    cfg = json.load(open(os.path.join(ROOT, "log_config.json")))
    assert cfg["version"] == 1 and "handlers" in cfg


def test_graft_entry_contract():
    import importlib.util
    spec = importlib.util.spec_from_file_location("graft_entry", os.path.join(ROOT, "__graft_entry__.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert callable(mod.build) and callable(mod.smoke)


def test_bench_cli_help():
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0
    for flag in ("--gpus", "--steps", "--warmup", "--profile"):
        assert flag in r.stdout
