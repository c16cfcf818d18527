"""bench.py's reporting helpers on the CPU: a secondary measurement that raises is reported in the
line and the run goes on (a failing cfg5 shard lost the whole bench line)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_secondary_failure_is_reported_and_the_run_goes_on():
    extra = {}

    def boom():
        raise RuntimeError("RCCL stand-in: rank 1 unreachable")

    assert bench.secondary(extra, "cfg5_shard", boom) is False
    assert "cfg5_shard" not in extra
    assert extra["cfg5_shard_error"] == "RuntimeError: RCCL stand-in: rank 1 unreachable"
    assert bench.secondary(extra, "cfg1", lambda: {"gibps": 1.0}) is True
    assert extra["cfg1"] == {"gibps": 1.0}
    # (a long message is cut to 300 characters: the line stays one line of JSON)
    bench.secondary(extra, "x", lambda: (_ for _ in ()).throw(ValueError("y" * 1000)))
    assert len(extra["x_error"]) == 300


def test_watchdog_exit_status_is_not_success():
    # the watchdog prints the partial line and exits with 3, not 0 (bench.py main: os._exit(3))
    src = open(bench.__file__).read()
    assert "os._exit(3)" in src and "os._exit(0)" not in src
