"""The bench line's `traffic` fields come from the PMC summaries committed for the current kernel
sources (profiles/pmc/config{3,cold}_<src_hash>.json, tools/gpu_pmc.sh).  These checks run on the
CPU: when a summary for these sources is committed, every leg's lookup must resolve (a kernel
renamed by a new template argument once left the line's traffic null without any error)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _summary(config):
    pmc, _ = bench.pmc_summary(config, bench.src_hash())
    if pmc is None:
        pytest.skip(f"no PMC summary committed for config {config} at sources {bench.src_hash()}: "
                    "the bench line's traffic will be null until tools/gpu_pmc.sh runs on them")
    return pmc


def test_name_match_template_arguments():
    k = "crane::k1_node_pass<4, 6, 256, true, false, 5, 0>(crane::K1Args, crane::K1Step)"
    assert bench.pmc_name_match(k, "crane::k1_node_pass", {3: "true", 4: "false"})
    assert not bench.pmc_name_match(k, "crane::k1_node_pass", {3: "false", 4: "false"})
    assert bench.pmc_name_match("crane::k3s_eval(crane::StepTables)", "crane::k3s_eval", {})
    assert not bench.pmc_name_match("crane::k3s_eval_x", "crane::k3s_eval", {})
    assert bench.pmc_name_match("crane::k3m_matrix<4, 6, 8, false, true, true>", "crane::k3m_matrix",
                                {-2: "true", -1: "true"})


def test_k2_path_traffic_picks_each_paths_kernels():
    ks = {"crane::k2l_partition<1024, 4096, true>": {"traffic_bytes": 10},
          "crane::k2l_partition<1024, 4096, false>": {"traffic_bytes": 20},
          "crane::k2y_bin_hist<2, 6>": {"traffic_bytes": 1},
          "crane::k2y_bin_hist<4, 5>": {"traffic_bytes": 2}}
    assert bench.k2_path_traffic(ks, True, 8_000_000) == 11    # 1,954 regions: two per lane
    assert bench.k2_path_traffic(ks, False, 16_000_000) == 22  # 3,907 regions: four per lane
    assert bench.k2_path_traffic(ks, False, 40_000_000) is None  # no k2y<8, ...> in the summary


def test_committed_summaries_resolve_every_leg():
    pmc3 = _summary("3")
    # the headline step's node pass: the streamed one beside the delta form's dense rows, the
    # record-holding one beside dedupe-form entries; the delta form's K2 + K3p launch
    assert (bench.pmc_traffic(pmc3, "k1_stream_steps") or bench.pmc_traffic(pmc3, "k1_node_pass+k3a_steps")) is not None
    assert (bench.pmc_traffic(pmc3, "k2_delta+k3p_pods") or bench.pmc_traffic(pmc3, "k2x_dedupe+k3p_pods")) is not None
    cold = _summary("cold")
    # the cold leg's step pass (bench.cold_leg: the streamed pass, else the fused one) and the
    # record-writing pass
    assert (bench.pmc_traffic(cold, "k1_stream_steps") or bench.pmc_traffic(cold, "k1_node_pass+k3a_steps")) is not None
    assert bench.pmc_traffic(cold, "k1_node_pass") is not None
    ks = cold["kernels"]
    n_read = 7_984_599  # the cold leg's ordered log: bindings inside the widest window
    assert bench.k2_path_traffic(ks, True, n_read) is not None
    assert bench.k2_path_traffic(ks, False, bench.COLD["bindings"]) is not None
    json.dumps(cold)
