"""bench.py's host-side plumbing on CPU: the torch-free dispatcher child
(bench.py dispatch_child: started before the bench touches a GPU, idle until
"go", never imports torch) and the parent's collection of its JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_dispatch_child_idle_exit_without_torch():
    # EOF on stdin (the parent died or ran --no-dispatch): the child exits 0
    # without a GPU call and without ever importing torch
    code = ("import io, sys; sys.argv = ['bench.py', '--dispatch-child', '--packets', '4096']; "
            "sys.stdin = io.StringIO(''); import bench; rc = bench.dispatch_child(bench.parse_args()); "
            "print(json.dumps({'rc': rc, 'torch': 'torch' in sys.modules}))")
    out = subprocess.run([sys.executable, "-c", "import json; " + code], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res == {"rc": 0, "torch": False}


def test_dispatch_child_result_parses_last_json_line():
    child = subprocess.Popen([sys.executable, "-c",
                              "import sys, json; assert sys.stdin.readline().strip() == 'go'; "
                              "print('noise'); print(json.dumps({'1': {'directional_pps': 1.0}}))"],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    assert bench.dispatch_child_result(child) == {"1": {"directional_pps": 1.0}}


def test_dispatch_child_result_reports_failure():
    child = subprocess.Popen([sys.executable, "-c", "import sys; sys.stdin.readline(); sys.exit('boom')"],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    res = bench.dispatch_child_result(child)
    assert "error" in res and "boom" in res["error"]


def test_dispatch_plan_shards_and_devices():
    ns = type("A", (), {"dispatch_shards": ""})()
    counts, devs_for = bench.dispatch_plan(ns, [0])
    assert counts == [1, 2, 4] and devs_for(4) == [0, 0, 0, 0]
    counts, devs_for = bench.dispatch_plan(ns, [0, 1, 2])
    assert counts == [3] and devs_for(3) == [0, 1, 2]
    ns.dispatch_shards = "2,5"
    counts, devs_for = bench.dispatch_plan(ns, [0, 1])
    assert counts == [2, 5] and devs_for(5) == [0, 1, 0, 1, 0]
