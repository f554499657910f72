"""bench.py's launcher decision (the driver's `python bench.py --gpus N` shape and its torchrun shape): with no
launcher and N > 1 the bench starts one worker per GPU itself; under a launcher WORLD_SIZE must equal --gpus."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.mark.parametrize("gpus,env,plan", [
    (1, {}, "run"),
    (2, {}, "spawn"),
    (8, {}, "spawn"),
    (8, {"WORLD_SIZE": "8"}, "run"),
    (1, {"WORLD_SIZE": "1"}, "run"),
    (2, {"WORLD_SIZE": "1"}, "mismatch"),
    (1, {"WORLD_SIZE": "4"}, "mismatch"),
    (0, {}, "mismatch"),
])
def test_launch_plan(gpus, env, plan):
    assert bench.launch_plan(gpus, env) == plan


def test_spawn_command_shape(monkeypatch):
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    rc = bench.spawn_workers(4, ["--gpus", "4", "--steps", "2"])
    assert rc == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"]
    assert os.path.basename(cmd[-5]) == "bench.py"


def test_mismatch_exits_nonzero_before_any_gpu_call():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2
    assert "WORLD_SIZE=3" in p.stderr


def test_profile_order_is_by_round_then_tag_length():
    """profiles/ summaries are picked newest-first by round tag, not by basename (r04t sorted after r04ae)."""
    names = ["r05ab_traffic.json", "r05b_traffic.json", "r04ae_traffic.json", "r04t_traffic.json", "r06a_traffic.json",
             "r05z_c5_traffic.json"]
    got = [os.path.basename(p) for p in sorted(names, key=bench.profile_order)]
    assert got == ["r04t_traffic.json", "r04ae_traffic.json", "r05b_traffic.json", "r05z_c5_traffic.json",
                   "r05ab_traffic.json", "r06a_traffic.json"]


@pytest.mark.parametrize("steps,warmup,extra", [
    (20, 5, 2),   # the driver's run: warmup ends alone in slot 0, the timed run alone in slot 1
    (5, 2, 3),    # the default: warmup met beside-slot-0 only
    (20, 4, 0),   # warmup already met every graph of the timed run
    (4, 4, 0),
    (1, 1, 0),
    (2, 1, 2),
    (3, 0, 0),    # no warmup: nothing to complete
])
def test_warmup_completion(steps, warmup, extra):
    assert bench.warmup_completion(steps, warmup) == extra


def test_warmup_completion_covers_every_timed_graph():
    for steps in range(1, 12):
        for warmup in range(1, 8):
            extra = bench.warmup_completion(steps, warmup)
            have = bench.decode_graph_keys(warmup) | bench.decode_graph_keys(extra)
            assert bench.decode_graph_keys(steps) <= have, (steps, warmup, extra)
            assert extra <= 4
