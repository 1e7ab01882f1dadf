"""The committed PMC summary matches this tree's kernel sources (CPU only).

bench.py reports `roofline.traffic` and the odd legs' `traffic` only from a
PMC summary collected on exactly the sources it hashes (bench.py
KERNEL_SOURCES / ODD_SOURCES, including tuning.h): an edit to any of them
after the last `scripts/final.sh first` silently drops those fields from
the driver's bench line.  This test makes that visible before the round ends.
"""
import bench


def test_headline_pmc_summary_is_fresh():
    data, path, why = bench.load_pmc()
    assert data is not None, why


def test_odd_pmc_summary_is_fresh():
    data, path, why = bench.load_pmc()
    assert data is not None, why
    assert data.get("odd_sources_sha256") == bench.kernel_sources_sha256(bench.ODD_SOURCES), (
        f"{path} was collected on other odd-kernel sources: rerun scripts/final.sh first")
    # the odd legs read these kernels' bytes from it (apply passes code their
    # guard bands inside the main kernel since round 6; Verify keeps the
    # separate guard-band launch)
    for name in ("gf_odd_edges<2, false, 128>", "gf_odd_planrec"):
        assert name in data["kernels"], name
    assert any(x.startswith("gf_odd_rec<") for x in data["kernels"])
    # each odd leg's bytes come from its own launches (bench.py leg markers)
    for leg in bench.PMC_LEGS:
        assert any(x.startswith("gf_odd") for x in data.get("legs", {}).get(leg, {})), leg
