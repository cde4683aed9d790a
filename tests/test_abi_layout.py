"""CPU: include/mccs_devcomm.h is layout-identical to the reference devcomm.h.

Golden numbers (tests/golden/abi_layout.json) were printed by
oracle/_ref/ref_layout, compiled from the reference header itself
(src/collectives/include/devcomm.h:36-163).
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "abi_layout.json")


def _run(exe):
    return json.loads(subprocess.run([exe], check=True, capture_output=True, text=True).stdout)


def _golden():
    with open(GOLDEN) as f:
        d = json.load(f)
    d.pop("_source", None)
    return d


def test_own_header_matches_golden():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "own_layout"], check=True)
    assert _run(os.path.join(ROOT, "oracle", "own_layout")) == _golden()


def test_reference_header_matches_golden():
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_layout")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built (reference tree absent)")
    assert _run(exe) == _golden()


def test_header_is_valid_c():
    r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                        "-x", "c", os.path.join(ROOT, "include", "mccs_devcomm.h")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_ctypes_mirror_layout():
    from mccs_amd import abi

    g = _golden()
    for name, size in abi.SIZES.items():
        assert g[f"sizeof({name})"] == size, name
    for (sname, field), off in abi.OFFSETS.items():
        assert g[f"{sname}.{field}"] == off, (sname, field)
