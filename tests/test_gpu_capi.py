"""The C-ABI from plain C (tests/capi/capi_allreduce.c, built with gcc -std=c11
by mccs_amd/build.py): communicator init, grouped AllReduce (the
allreduce_proto int32 known answer and an exact-sum fp32 case) and the
standalone chunk reduce, with no Python in the data path."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "capi", "capi_allreduce")


@pytest.mark.gpu
def test_c_driver_runs():
    """Also section 5: a stream destroyed with an
    AllReduce still queued, a new stream at the same address, an AllReduce on
    it at once.  Under the runtime a C / Rust caller links (ROCm 7.2, no
    torch) the library tells streams apart by hipStreamGetId, so it orders the
    second launch after the first on the host: both exact, and the launch
    guard never saw them overlap."""
    assert os.path.exists(BIN), "build it with __graft_entry__.build() / python -m mccs_amd.build"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "capi ok" in r.stdout, r.stdout + r.stderr
    assert "stream ids: native" in r.stdout, r.stdout  # the id branch, not the address fallback
    assert "guard waits: 0" in r.stdout, r.stdout


def test_header_is_plain_c11():
    """include/mccs_hip.h compiles as C11 next to the HIP C runtime header
    (the bindgen / cgo view of the boundary); no GPU needed."""
    from mccs_amd import build as b

    r = subprocess.run(b.capi_cmd(b.CAPI_SRC, "", syntax_only=True), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
