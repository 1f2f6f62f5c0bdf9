"""bench.py --gpus N without an external launcher (CPU): the launch decision, the child
torch.distributed.run command, the relay of rank 0's JSON line, and the refusal of a WORLD_SIZE that
contradicts --gpus (so a driver's ``bench.py --gpus 8`` can never report one rank)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("gpus, env, want", [
    (1, {}, ("run", 1)),
    (8, {}, ("spawn", 8)),
    (2, {"WORLD_SIZE": ""}, ("spawn", 2)),
    (8, {"WORLD_SIZE": "8"}, ("run", 8)),
    (1, {"WORLD_SIZE": "1"}, ("run", 1)),
    (8, {"WORLD_SIZE": "1"}, "error"),   # a launcher that started one rank for an 8-GPU job
    (1, {"WORLD_SIZE": "4"}, "error"),
    (0, {}, "error"),
    (2, {"WORLD_SIZE": "two"}, "error"),
])
def test_bench_launch_plan(gpus, env, want):
    plan = _bench_module().launch_plan(gpus, env)
    if want == "error":
        assert plan[0] == "error" and plan[1]
    else:
        assert plan == want


def test_bench_spawn_command_is_one_node_torchrun():
    cmd = _bench_module().spawn_command(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_bench_spawn_ranks_relays_rank0_line(tmp_path, monkeypatch, capsys):
    """spawn_ranks starts a real torch.distributed.run child (2 CPU ranks running a stand-in script that
    does what bench.py's ranks do with the env: rank 0 prints the line) and relays its stdout."""
    script = tmp_path / "rank.py"
    script.write_text("import json, os\n"
                      "if os.environ['RANK'] == '0':\n"
                      "    print(json.dumps({'n_gpus': int(os.environ['WORLD_SIZE'])}), flush=True)\n")
    bench = _bench_module()
    real = bench.spawn_command
    monkeypatch.setattr(bench, "spawn_command", lambda g, argv, port: real(g, argv, port)[:-1 - len(argv)] + [str(script)])
    rc = bench.spawn_ranks(2, [])
    out = capsys.readouterr().out
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert rc == 0 and len(lines) == 1 and json.loads(lines[0]) == {"n_gpus": 2}


def test_bench_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="1")
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=120)
    assert res.returncode == 2 and "WORLD_SIZE=1" in res.stderr and not res.stdout.strip()
