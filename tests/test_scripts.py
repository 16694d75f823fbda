"""Static checks of the launch scripts and repo contracts (reference: test_run_sh.py)."""
import json
import os
import stat
import sys

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


def test_bench_gemma_config_uses_fused_engine_and_gemma_layers():
    """The Gemma-3 1B bench config runs the fused engine (lowered to the Gemma executor)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    args = bench.parse_args(["--model", "gemma3-1b"])
    assert args.engine == "fused" and args.batch == 64 and args.seq == 1024
    assert bench.parse_args([]).engine == "fused"
    layers = bench.gemma3_1b_layers(2)
    names = [next(iter(l)) for l in layers]
    assert names.count("transformerblock") == 2 or "rmsnorm" in names, names


def _run_bench(args, env_extra=None, timeout=300):
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.slow
def test_bench_self_launches_ranks_cpu_gloo():
    """`python bench.py --gpus 2` (no torchrun) spawns 2 ranks itself; rank 0 prints ONE JSON line
    with n_gpus == 2 and the communicator's view of the group (2-rank gloo rehearsal)."""
    r = _run_bench(["--gpus", "2", "--device", "cpu", "--model", "tiny", "--steps", "2", "--warmup", "1",
                    "--nocomm-steps", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 2 * d["config"]["micro_batch_per_gpu"]
    assert d["comm"]["nranks"] == 2 and d["comm"]["transport"] == "gloo" and d["comm"]["buckets"] >= 1
    assert d["comm"]["allreduce_exposed_ms"] >= 0.0
    assert d["comm"]["probe_allreduce_mb"] == 4 and d["comm"]["probe_busbw_GBps"] > 0
    assert d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    # first-contact record: both ranks' devices, the checked sweep, the transport choice
    assert len(d["comm"]["devices"]) == 2
    sweep = d["comm"]["sweep"]
    assert {r["bucket_mb"] for r in sweep} == {1, 4} and {r["wire"] for r in sweep} == {"fp32", "bf16"}
    assert all(r["ok"] and r["busbw_GBps"] > 0 and r["transport"] == "c10d" for r in sweep)
    assert all(r["channels"] is None and r["proto"] is None and r["algo"] is None for r in sweep)  # arm keys
    pl = d["comm"]["plan"]
    assert pl["transport"] == "c10d" and pl["wire"] == "fp32" and pl["channels"] is None and pl["proto"] is None
    assert pl["algo"] is None
    assert pl["grad_bytes"] > 0 and pl["backward_ms_estimate"] is None and "predicted_fp32_ms" in pl
    assert set(d["comm"]["rccl"]) == {"coll_channels", "nranks", "log"}
    assert pl["agreed_ranks"] == 2 and pl["applied_env"] == {"PENROZ_COMM": "c10d"}
    st = d["comm"]["sweep_stats"]
    assert st["arms_run"] == ["c10d"] and not st["arms_skipped"] and not st["arms_failed"]
    assert 0 < st["wall_s"] <= st["budget_s"]


def test_bench_refuses_more_gpus_than_visible():
    """No silent 1-GPU number for `--gpus 2` on a box with fewer devices (here: none)."""
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], timeout=120)
    assert r.returncode != 0
    assert "GPU(s) are visible" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_comm_choice_rules():
    from penroz.parallel.commtune import choose
    row = lambda tr, bw, ok=True, mb=64, wire="fp32": {"transport": tr, "wire": wire, "bucket_mb": mb,
                                                        "busbw_GBps": bw, "ok": ok}
    assert choose([row("c10d", 100), row("native", 120)], 64)["transport"] == "native"
    assert choose([row("c10d", 100), row("native", 101)], 64)["transport"] == "c10d"   # inside the margin
    assert choose([row("c10d", 100), row("native", 200, ok=False)], 64)["transport"] == "c10d"  # wrong sum
    assert choose([row("c10d", 100)], 64)["transport"] == "c10d"
    # nearest swept size to the reducer's bucket decides
    rows = [row("c10d", 100, mb=32), row("native", 90, mb=32), row("c10d", 100, mb=128), row("native", 150, mb=128)]
    assert choose(rows, 100)["transport"] == "native" and choose(rows, 40)["transport"] == "c10d"


def _prow(tr, mb, bw, ok=True, wire="fp32", ch=None, proto="", algo=""):
    # busbw at world 8 = algbw * 2 * 7 / 8
    return {"transport": tr, "channels": ch if tr == "native" else None, "proto": proto if tr == "native" else None,
            "algo": algo if tr == "native" else None, "wire": wire, "bucket_mb": mb, "busbw_GBps": bw,
            "algbw_GBps": bw * 8 / 14, "ok": ok}


def test_comm_plan_judges_each_transport_at_its_own_bucket():
    """the transport is compared at each arm's own chosen bucket size, not at a fixed 64 MB."""
    from penroz.parallel.commtune import plan
    rows = [_prow("c10d", 16, 100), _prow("c10d", 64, 104),
            _prow("native", 16, 70, ch=0), _prow("native", 64, 130, ch=0)]
    p = plan(rows, grad_bytes=652 * 2**20)
    # c10d's size is 16 MB (within 90 % of its best), native's 64 MB: 130 vs 100 -> native at 64 MB
    assert p["transport"] == "native" and p["bucket_mb"] == 64 and p["channels"] == 0
    rows = [_prow("c10d", 16, 120), _prow("native", 16, 70, ch=0), _prow("native", 64, 121, ch=0)]
    assert plan(rows, grad_bytes=1)["transport"] == "c10d"  # inside the 3 % margin
    rows = [_prow("c10d", 16, 120), _prow("native", 64, 300, ok=False, ch=0)]
    assert plan(rows, grad_bytes=1)["transport"] == "c10d"  # wrong sums never win


def test_comm_plan_picks_channel_count():
    """The channel count comes with the winning native arm (NCCL_MIN/MAX_NCHANNELS)."""
    from penroz.parallel.commtune import plan
    rows = [_prow("c10d", 64, 100), _prow("native", 64, 110, ch=0), _prow("native", 64, 160, ch=16),
            _prow("native", 64, 140, ch=32), _prow("native", 32, 170, ok=False, ch=8)]
    p = plan(rows, grad_bytes=652 * 2**20)
    assert p["transport"] == "native" and p["channels"] == 16 and p["busbw_GBps"] == 160
    assert "16 channels" in p["reason"]


def test_comm_plan_picks_protocol():
    """A forced protocol (the per-communicator NCCL_PROTO) comes with the winning native arm; a
    protocol arm with wrong sums never wins; the bf16 wire is looked up on the winning arm."""
    from penroz.parallel.commtune import plan
    rows = [_prow("c10d", 64, 100), _prow("native", 64, 120, ch=0), _prow("native", 64, 150, ch=0, proto="Simple"),
            _prow("native", 64, 190, ch=0, proto="LL128", ok=False), _prow("native", 64, 140, ch=16)]
    p = plan(rows, grad_bytes=652 * 2**20)
    assert p["transport"] == "native" and p["channels"] == 0 and p["proto"] == "Simple" and p["busbw_GBps"] == 150
    assert "protocol Simple" in p["reason"]
    rows.append(_prow("native", 64, 150, ch=0, proto="Simple", wire="bf16"))
    g = 6550 * 2**20
    assert plan(rows, g, backward_ms=1.0, auto_bf16=True)["wire"] == "bf16"
    # RCCL's own protocol choice wins when nothing forced beats it
    rows = [_prow("c10d", 64, 100), _prow("native", 64, 160, ch=0), _prow("native", 64, 150, ch=0, proto="LL128")]
    assert plan(rows, grad_bytes=1)["proto"] == ""


def test_comm_plan_picks_algorithm():
    """A forced algorithm (the per-communicator NCCL_ALGO) comes with the winning native arm, never
    mixed with another arm's protocol; wrong sums never win; RCCL's own choice wins ties."""
    from penroz.parallel.commtune import plan
    rows = [_prow("c10d", 64, 100), _prow("native", 64, 120, ch=0), _prow("native", 64, 130, ch=0, proto="Simple"),
            _prow("native", 64, 155, ch=0, algo="Ring"), _prow("native", 64, 200, ch=0, algo="Tree", ok=False)]
    p = plan(rows, grad_bytes=652 * 2**20)
    assert p["transport"] == "native" and p["algo"] == "Ring" and p["proto"] == "" and p["busbw_GBps"] == 155
    assert "algorithm Ring" in p["reason"]
    rows = [_prow("c10d", 64, 100), _prow("native", 64, 160, ch=0), _prow("native", 64, 150, ch=0, algo="Tree")]
    assert plan(rows, grad_bytes=1)["algo"] == ""
    # the bf16 wire is looked up on the winning (channels, protocol, algorithm) arm only
    rows = [_prow("c10d", 64, 100), _prow("native", 64, 155, ch=0, algo="Ring"),
            _prow("native", 64, 150, ch=0, wire="bf16")]
    assert plan(rows, 6550 * 2**20, backward_ms=1.0, auto_bf16=True)["wire"] == "fp32"


def test_comm_plan_bf16_wire_only_when_exposed():
    """bf16 wire recommended only when the predicted fp32 all-reduce of the whole gradient exceeds
    the backward and the bf16 arm is correct and clearly faster; APPLIED only with auto_bf16 (ADVICE
    r4: the default wire stays the reference DDP's fp32)."""
    from penroz.parallel.commtune import plan
    rows = [_prow("c10d", 64, 100), _prow("c10d", 64, 100, wire="bf16")]
    g = 6550 * 2**20  # GPT-2 XL fp32 gradients
    fp32_ms = g / (100 * 8 / 14 * 1e9) * 1e3
    P = lambda r, **kw: plan(r, g, auto_bf16=True, **kw)
    assert P(rows, backward_ms=fp32_ms * 2)["wire"] == "fp32"     # hidden behind the backward
    p = P(rows, backward_ms=fp32_ms / 2)
    assert p["wire"] == "bf16" and abs(p["predicted_bf16_ms"] * 2 - p["predicted_fp32_ms"]) < 0.01
    assert P(rows, backward_ms=None)["wire"] == "fp32"            # no estimate, no change
    bad = [_prow("c10d", 64, 100), _prow("c10d", 64, 100, wire="bf16", ok=False)]
    assert P(bad, backward_ms=1.0)["wire"] == "fp32"              # wrong bf16 sums
    slow = [_prow("c10d", 64, 100), _prow("c10d", 64, 40, wire="bf16")]
    assert P(slow, backward_ms=1.0)["wire"] == "fp32"             # bf16 not faster overall
    assert plan([], g)["transport"] == "c10d"
    # default: recorded, never applied
    q = plan(rows, g, backward_ms=fp32_ms / 2)
    assert q["wire"] == "fp32" and q["wire_recommendation"] == "bf16"
    assert plan(rows, g, backward_ms=fp32_ms * 2)["wire_recommendation"] == "fp32"


def test_parse_rccl_log_nranks_and_channels():
    """rccl.nranks / coll_channels come from what RCCL itself logged at init."""
    from penroz.parallel.commtune import parse_rccl_log
    text = ("host:1:1 [0] NCCL INFO Channel 00/16 :    0   1   2   3   4   5   6   7\n"
            "host:1:1 [0] NCCL INFO 16 coll channels, 16 collnet channels, 0 nvls channels\n"
            "host:1:1 [0] NCCL INFO comm 0x5581 rank 0 nranks 8 cudaDev 0 busId 5000 - Init COMPLETE\n")
    assert parse_rccl_log(text) == {"coll_channels": 16, "nranks": 8}
    assert parse_rccl_log("nothing here") == {"coll_channels": None, "nranks": None}
    assert parse_rccl_log("ncclCommInitRank comm 0x1 rank 3 nRanks 4 nNodes 1")["nranks"] == 4


def test_sweep_arms_default_is_rccl_only(monkeypatch):
    """the forced channel / protocol / algorithm arms are opt-in."""
    from penroz.parallel import commtune
    monkeypatch.delenv("PENROZ_COMM_SWEEP_ARMS", raising=False)
    assert commtune.sweep_arms() == ((0,), ("",), ("",))
    monkeypatch.setenv("PENROZ_COMM_SWEEP_ARMS", "full")
    assert commtune.sweep_arms() == (commtune.SWEEP_CHANNELS, commtune.SWEEP_PROTOS, commtune.SWEEP_ALGOS)


def test_comm_plan_identical_for_identical_rows():
    """The plan is a pure function of the (MAX/MIN-reduced, hence identical) sweep rows: shuffled row
    order on another rank gives the same plan."""
    import random
    from penroz.parallel.commtune import plan
    rows = [_prow("c10d", mb, 90 + mb / 8) for mb in (16, 32, 64, 128)] + \
           [_prow("native", mb, 80 + mb / 4, ch=0) for mb in (16, 32, 64, 128)] + \
           [_prow("c10d", 64, 120, wire="bf16"), _prow("native", 64, 130, ch=0, wire="bf16")]
    ref = plan(rows, 652 * 2**20, backward_ms=3.0)
    for seed in range(5):
        r = list(rows)
        random.Random(seed).shuffle(r)
        assert plan(r, 652 * 2**20, backward_ms=3.0) == ref


def test_comm_bucket_choice_rule(monkeypatch):
    """Smallest swept bucket within 90 % of the best bus bandwidth of the chosen transport; wrong
    sums and other transports / wires are ignored; the reducer reads the chosen size at call time."""
    from penroz.parallel.commtune import choose_bucket
    from penroz.parallel import reducer as R
    row = lambda tr, mb, bw, ok=True, wire="fp32": {"transport": tr, "wire": wire, "bucket_mb": mb,
                                                     "busbw_GBps": bw, "ok": ok}
    rows = [row("c10d", 16, 60), row("c10d", 32, 88), row("c10d", 64, 95), row("c10d", 128, 100),
            row("c10d", 256, 99), row("native", 16, 150, ok=False), row("c10d", 16, 200, wire="bf16")]
    c = choose_bucket(rows, "c10d")
    assert c["bucket_mb"] == 64 and c["best_busbw_GBps"] == 100
    assert choose_bucket(rows, "native") is None
    monkeypatch.setenv("PENROZ_BUCKET_MB", "32")
    assert R.default_bucket_mb("nccl") == 32.0 and R.default_bucket_mb("gloo") == 32.0
    monkeypatch.delenv("PENROZ_BUCKET_MB")
    assert R.default_bucket_mb("gloo") == R.GLOO_BUCKET_MB and R.default_bucket_mb("nccl") == R.DEFAULT_BUCKET_MB


def test_init_group_passes_timeout(monkeypatch):
    import datetime
    import torch.distributed as dist
    from penroz.parallel import dist as pdist
    seen = {}
    monkeypatch.setattr(dist, "is_initialized", lambda: False)
    monkeypatch.setattr(dist, "init_process_group", lambda **kw: seen.update(kw))
    monkeypatch.setenv("PENROZ_DIST_TIMEOUT", "42")
    monkeypatch.delenv("TORCH_NCCL_ASYNC_ERROR_HANDLING", raising=False)
    import torch
    pdist.init_group("nccl", torch.device("cuda", 0))
    assert seen["timeout"] == datetime.timedelta(seconds=42) and seen["backend"] == "nccl"
    assert seen["device_id"] == torch.device("cuda", 0)
    assert os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] == "1"
    seen.clear()
    pdist.init_process_group("cpu")
    assert seen["backend"] == "gloo" and "device_id" not in seen and seen["timeout"].total_seconds() == 42


@pytest.mark.slow
def test_stalled_rank_fails_within_timeout():
    """A rank stuck outside a collective makes its peer fail after PENROZ_DIST_TIMEOUT, and the
    supervising launcher ends the whole group with a nonzero code: no hang."""
    import subprocess
    import sys
    import time
    code = ("import sys, types, bench; sys.exit(bench.launch_ranks(types.SimpleNamespace(gpus=2, device='cpu'), [], "
            f"script={os.path.join(ROOT, 'tests', 'stall_rank_helper.py')!r}))")
    env = dict(os.environ, PENROZ_DIST_TIMEOUT="3")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=90, env=env)
    took = time.time() - t0
    assert r.returncode != 0, r.stdout + r.stderr
    assert "rank0 collective failed" in r.stdout, r.stdout + r.stderr
    assert took < 60, took


@pytest.mark.slow
def test_bench_rank_failure_stops_group():
    """A failing rank ends the self-launched group with a nonzero exit code (no hang)."""
    r = _run_bench(["--gpus", "2", "--device", "cpu", "--model", "tiny", "--steps", "1", "--warmup", "0",
                    "--seq", "4096"], timeout=120)
    assert r.returncode != 0


def test_ab_tool_arms_and_workloads():
    """bench/ab.py: arm specs parse to env dicts; every workload kind maps to a bounded command."""
    sys.path.insert(0, os.path.join(ROOT, "bench"))
    import ab
    assert ab.parse_arm("base:PENROZ_EXT_DIR=build_ab X=1") == ("base", {"PENROZ_EXT_DIR": "build_ab", "X": "1"})
    assert ab.parse_arm("new:") == ("new", {})
    with pytest.raises(SystemExit):
        ab.parse_arm("bad:NOVALUE")
    cmd, lim = ab.work_cmd("headline", 20, 5)
    assert cmd[1:] == ["bench.py", "--steps", "20", "--warmup", "5", "--ref-steps", "0"] and lim > 0
    assert ab.work_cmd("gemma3-1b:8", 20, 5)[0][-2:] == ["--batch", "8"]
    assert ab.work_cmd("decode:gpt2:1", 20, 5)[0][-4:] == ["--model", "gpt2", "--batch", "1"]
    assert "--D" in ab.work_cmd("attn:--B 4 --D 64", 20, 5)[0]
    assert ab.headline_number('noise\n{"ms_per_step": 61.2, "value": 1.0, "x": 3}\n') == {"ms_per_step": 61.2, "value": 1.0}


def test_bench_gemma4_config_shapes():
    """The Gemma-4-class bench config: alternating D = 256 sliding / D = 512 full-attention layers,
    double-wide MLPs on the KV-shared tail; it lowers to the fused Gemma executor and the gradient
    plan counts its parameters."""
    import torch
    import bench
    from penroz.models.gemma_executor import GemmaExecutor
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    cfg = bench.MODELS["gemma4-e2b"]
    shapes = bench.gemma_layer_shapes(cfg)
    assert shapes[0] == (256, 1, 6144) and shapes[1] == (512, 1, 6144) and shapes[-1] == (512, 1, 12288)
    with torch.device("meta"):
        m = NeuralNetworkModel("g4", Mapper(Mapper.from_hf_config(bench.gemma4_config(cfg)), {"adamw": {}}))
    spec = GemmaExecutor.match(m)
    assert spec is not None and [(b.D, b.Hkv, b.F) for b in spec.blocks] == shapes
    args = bench.parse_args(["--model", "gemma4-e2b", "--batch", "8"])
    grad_bytes, _ = bench._grad_plan_inputs(args)
    assert grad_bytes == 4 * sum(p.numel() for p in m.parameters())


def test_gemm_table_guard_keeps_only_a_faster_table(monkeypatch):
    """the shipped GEMM table is timed against hipBLASLt's heuristic before the
    timed region and dropped when slower; the choice is left switched on."""
    import torch.cuda.tunable as tunable
    from penroz.ops import gemm as G
    state = {}
    monkeypatch.setattr(tunable, "enable", lambda on=True: state.__setitem__("on", on))
    monkeypatch.setattr(G, "_tuned_state", {"loaded": True})
    times = {True: 0.060, False: 0.063}
    r = G.guard_tuned_gemms(lambda n: times[state["on"]] * n, steps=3)
    assert r["table_kept"] and state["on"] is True and r["with_table_ms"] == 60.0 and r["heuristic_ms"] == 63.0
    times = {True: 0.0645, False: 0.0635}
    r = G.guard_tuned_gemms(lambda n: times[state["on"]] * n, steps=3)
    assert not r["table_kept"] and state["on"] is False
    monkeypatch.setattr(G, "_tuned_state", {})
    assert G.guard_tuned_gemms(lambda n: 1.0) == {}


@pytest.mark.slow
@pytest.mark.parametrize("world", [4, 8])
def test_bench_multi_rank_cpu_matches_single_process(world):
    """the data-parallel bench at 4 and 8 ranks (gloo on the CPU, tiny model).
    Every rank agrees on the first-contact plan and builds the same gradient buckets, and the
    rank-averaged loss and the parameters after the run equal one process training on the
    concatenated batches (``--data-ranks``)."""
    common = ["--device", "cpu", "--model", "tiny", "--steps", "3", "--warmup", "1", "--nocomm-steps", "0",
              "--comm-probe-iters", "2"]
    r = _run_bench(["--gpus", str(world)] + common, env_extra={"OMP_NUM_THREADS": "1"}, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == world and d["comm"]["nranks"] == world
    assert d["comm"]["plan"]["agreed_ranks"] == world and d["comm"]["bucket_plans_agree"] == world
    assert len(d["comm"]["devices"]) == world
    s = _run_bench(["--gpus", "1", "--batch", str(4 * world), "--data-ranks", str(world)] + common,
                   env_extra={"OMP_NUM_THREADS": "4"}, timeout=600)
    assert s.returncode == 0, s.stderr[-3000:]
    one = _json_line(s.stdout)
    assert one["config"]["global_batch"] == d["config"]["global_batch"]
    assert abs(d["final_loss_global"] - one["final_loss"]) <= 1e-4 * abs(one["final_loss"]), (d, one)
    assert abs(d["param_checksum"] - one["param_checksum"]) <= 1e-4 * one["param_checksum"]


def test_split_last_bucket_and_ready_map():
    """The embedding bucket (produced by the backward's last kernel) is cut into pieces that all
    become ready with the last segment; every bucket is launched exactly once."""
    from penroz.parallel.reducer import plan_buckets, ready_map, split_last_bucket
    segs = [(0, 1000), (1000, 1300), (1300, 1600), (1600, 1900), (1900, 6000)]
    b = plan_buckets(segs, 600 * 4)
    assert b == [(0, 1000), (1000, 1600), (1600, 6000)]
    s4 = split_last_bucket(b, 4, align=64)
    assert s4[:2] == b[:2] and s4[2][0] == 1600 and s4[-1][1] == 6000 and len(s4) == 2 + 4
    assert all(x[1] == y[0] for x, y in zip(s4, s4[1:]))
    assert all((e - s) % 64 == 0 for s, e in s4[2:-1])
    rm = ready_map(s4, segs)
    assert rm == {0: [0], 2: [1], 4: [2, 3, 4, 5]}
    assert sorted(i for v in rm.values() for i in v) == list(range(len(s4)))
    assert split_last_bucket(b, 1) == b
