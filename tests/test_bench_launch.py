"""bench.py's launch logic: `--gpus N` without a launcher starts N ranks through
torch.distributed.run as a child process; under a launcher `--gpus` must equal WORLD_SIZE.  CPU only:
the decisions are taken before anything touches a GPU, and `--dry-run` prints them."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def _run(args, **kw):
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=300, env=_env(**kw))


def test_gpus_n_spawns_torchrun_child():
    r = _run(["--gpus", "2", "--steps", "5", "--warmup", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    i = cmd.index(BENCH)
    assert cmd[i + 1:] == ["--gpus", "2", "--steps", "5", "--warmup", "2"]   # same args, no --dry-run


def test_single_gpu_runs_in_process():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["launch"] is None and d["world_size"] == 1


def test_under_launcher_gpus_must_match_world_size():
    r = _run(["--gpus", "4", "--dry-run"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    r = _run(["--gpus", "2", "--dry-run"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"launch": None, "world_size": 2}


def test_launch_plan_unit():
    # import only the launch helpers: executing the module body past them would import orbx
    src = open(BENCH).read().split('\nif __name__ == "__main__":\n')[0]
    ns = {"__file__": BENCH, "__name__": "bench_launch"}
    exec(compile(src, BENCH, "exec"), ns)
    assert ns["launch_plan"]([], {}) == ("run", 1)
    assert ns["launch_plan"](["--gpus", "1"], {}) == ("run", 1)
    assert ns["launch_plan"]([], {"WORLD_SIZE": "8"}) == ("run", 8)
    assert ns["launch_plan"](["--gpus=8"], {"WORLD_SIZE": "8"}) == ("run", 8)
    assert ns["launch_plan"](["--gpus", "0"], {})[0] == "error"
    mode, cmd = ns["launch_plan"](["--gpus", "8"], {})
    assert mode == "spawn" and "--nproc-per-node=8" in cmd


def test_spawn_relays_json_line_and_status(capfd):
    src = open(BENCH).read().split('\nif __name__ == "__main__":\n')[0]
    ns = {"__file__": BENCH, "__name__": "bench_launch"}
    exec(compile(src, BENCH, "exec"), ns)
    child = [sys.executable, "-c", "import sys; print('rank log'); print('{\"metric\": \"m\", \"value\": 1}'); sys.exit(3)"]
    assert ns["spawn_ranks"](child) == 3
    out, err = capfd.readouterr()
    assert out.strip() == '{"metric": "m", "value": 1}'
    assert "rank log" in err


def test_gpus_n_refused_without_that_many_gpus():
    # with fewer GPUs than --gpus the launcher refuses instead of starting ranks that would fail; the count
    # comes from sysfs and the *_VISIBLE_DEVICES lists, never from a HIP call
    r = _run(["--gpus", "2"], ROCR_VISIBLE_DEVICES="0")
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr


def test_visible_gpu_count_from_sysfs(tmp_path):
    src = open(BENCH).read().split('\nif __name__ == "__main__":\n')[0]
    ns = {"__file__": BENCH, "__name__": "bench_launch"}
    exec(compile(src, BENCH, "exec"), ns)
    count = ns["visible_gpu_count"]
    nodes = tmp_path / "nodes"
    for i, gfx in enumerate([0, 90500, 90500, 90500]):      # node 0: the CPU
        (nodes / str(i)).mkdir(parents=True)
        (nodes / str(i) / "properties").write_text("cpu_cores_count 4\ngfx_target_version %d\n" % gfx)
    assert count({}, str(nodes)) == 3
    assert count({"HIP_VISIBLE_DEVICES": "1"}, str(nodes)) == 1
    assert count({"ROCR_VISIBLE_DEVICES": "0,1,2,3,4"}, str(nodes)) == 3
    assert count({}, str(tmp_path / "absent")) is None
    assert count({"CUDA_VISIBLE_DEVICES": "0,1"}, str(tmp_path / "absent")) == 2
