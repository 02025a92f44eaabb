"""Object lifetimes of the C-ABI (include/odpg.h "object lifetimes"):
tables, counters, forwarders and fences may be destroyed in any order
relative to each other and to their context. Counters, forwarders and fences
hold a reference to the context, so destroying the context first leaves
them usable until their own destroy (round 4's counted run of
tools/wave_times.py died with SIGSEGV in teardown, gpurun_out/r04c; the
counters' destroy then read the context it was created on). Each order runs
in its own child process (tests/destroy_order_child.py), after counted
launches, and must exit 0."""
import itertools
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _orders():
    out = []
    for perm in itertools.permutations(["cnt", "tbl", "ctx"]):
        # fence and forwarder before everything, and after everything
        out.append(["fwd", "fence"] + list(perm))
        out.append(list(perm) + ["fence", "fwd"])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("order", _orders(), ids=lambda o: "-".join(o))
def test_destroy_in_any_order(order):
    r = subprocess.run([sys.executable, os.path.join(HERE, "destroy_order_child.py"),
                        ",".join(order)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, (order, r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert r.stdout.startswith("ok"), r.stdout
