"""bench.py's watchdog around the optional row-partitioned leg (CPU): a leg that returns in time
gives its value; a stalled one lets the line print and the process exit with status 3
(bench.WATCHDOG_EXIT), not 0, so a hang is visible to whoever checks the exit status."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_run_guarded_returns_value():
    sys.path.insert(0, REPO)
    import bench
    assert bench.run_guarded(lambda: 42, 30.0, lambda: None) == 42


def test_run_guarded_timeout_prints_and_exits():
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.run_guarded(lambda: time.sleep(60), 0.5, lambda: print('LINE', flush=True)); "
            "print('NOT REACHED')" % REPO)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert "LINE" in p.stdout and "NOT REACHED" not in p.stdout
