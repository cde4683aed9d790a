"""CPU: host-side helpers of the multi-GPU bench leg (mccs_amd/ring_bench.py)."""
import pytest

from mccs_amd import comm as C
from mccs_amd import ring_bench as rb


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
def test_default_rings_use_distinct_links(n):
    """Each default ring sends on a different outgoing link where the node has
    enough (2 x floor((n-1)/2) edge-disjoint directed cycles)."""
    rings = C.default_rings(n)
    for r in range(n):
        links = rb._out_links(rings, r)
        assert links == min(n - 1, len(rings)) or (n == 2 and links == 1), (n, r, links, rings)


def test_setup2_job_split():
    assert rb.setup2_jobs(8, False) == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert rb.setup2_jobs(8, True) == [[0, 2, 4, 6], [1, 3, 5, 7]]
    with pytest.raises(ValueError):
        rb.setup2_jobs(3, False)


def test_setup2_shapes_match_workload_files():
    # workloads/setup-2_vgg.toml: 574,668,960 B fp16; setup-2_gpt_1.toml: 83,886,080 B fp16
    assert [c * 2 for _, c in rb.SETUP2_JOBS] == [574_668_960, 83_886_080]


def test_workload_labels():
    assert rb.WORKLOADS[("float32", 128)].endswith("configs[2]")
    assert rb.WORKLOADS[("float16", 1024)].endswith("configs[3]")
