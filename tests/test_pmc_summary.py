"""scripts/pmc_summary.py maps mangled kernel names to the kernels the bench line reports (CPU):
longer names win over their prefixes (k_rp_build3 / k_rp_build, k_nagg_mains / k_nagg) and template
instantiations stay apart."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "scripts", "pmc_summary.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_kernel_name_mapping():
    m = _mod()
    ns = "hj3d::(anonymous namespace)::"
    assert m.short(ns + "k_rp_build3(HIP_vector_type<unsigned int, 2u> const*, unsigned int const*)") == "k_rp_build3"
    assert m.short(ns + "k_rp_build(HIP_vector_type<unsigned int, 2u> const*)") == "k_rp_build"
    assert m.short(ns + "k_nagg_mains(HIP_vector_type<unsigned int, 4u> const*)") == "k_nagg_mains"
    assert m.short(ns + "k_nagg(HIP_vector_type<unsigned int, 2u> const*, unsigned int const*)") == "k_nagg"
    assert m.short("void " + ns + "k_pk_probe<1, false>(HIP_vector_type<unsigned int, 2u> const*)") == \
        "k_pk_probe<1, false>"
    assert m.short("void " + ns + "k_rp_part1r<1024, 8, 16, true, false>(hj3d::RelView)").startswith("k_rp_part1")
    assert m.short(ns + "k_scan_lb(unsigned int const*)") is None
