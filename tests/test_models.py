"""Model registry + roofline generator parity with the reference's tables.

Golden values are the reference's shipped model_stats/*_16_bfloat16.txt
lines (Model_Size, Non_Expert_size, Average_Forward_Time, FFN time, Seq_len,
Embedded_dim); when /root/reference is mounted every one of its 72 files is
also compared field by field.
"""
import glob
import os

import pytest

from dlnetbench_amd.models import MODELS, compute_stats, get_model
from dlnetbench_amd.utils.stats import load_stats, parse_stats_text

GOLDEN_16_BF16 = {
    # model: (Model_Size, Non_Expert_size, fwd_us, ffn_fwd_us, Seq_len, Embedded_dim)
    "gpt2_l": (774030080, 0, 11682.31, 6871.95, 1024, 1280),
    "gpt2_xl": (1557611200, 0, 23765.49, 14316.56, 1024, 1600),
    "llama3_70b": (70553706496, 0, 8131499.33, 4378499.64, 8192, 8192),
    "llama3_8b": (8030261248, 0, 938249.92, 437849.96, 8192, 4096),
    "minerva_7b": (7399542784, 0, 406574.97, 218924.98, 4096, 4096),
    "mixtral_8x7b": (46702792704, 1700000000, 8506799.30, 3502799.71, 32768, 4096),
    "vit_b": (86389248, 0, 248.14, 158.65, 197, 768),
    "vit_h": (632404480, 0, 2376.55, 1533.06, 257, 1280),
    "vit_l": (304351232, 0, 873.24, 564.07, 197, 1024),
}


@pytest.mark.parametrize("name", sorted(GOLDEN_16_BF16))
def test_roofline_matches_reference_golden(name):
    size, ne, fwd, ffn, seq, d = GOLDEN_16_BF16[name]
    st = compute_stats(get_model(name), 16, "bfloat16", "b200")
    assert st.model_size == size
    assert st.non_expert_size == ne
    assert round(st.fwd_us, 2) == pytest.approx(fwd, abs=0.011)
    assert round(st.bwd_us, 2) == pytest.approx(2 * fwd, abs=0.021)
    assert round(st.ffn_fwd_us, 2) == pytest.approx(ffn, abs=0.011)
    assert st.seq_len == seq and st.hidden == d


def test_float8_halves_compute_bound_times():
    a = compute_stats(get_model("llama3_8b"), 16, "bfloat16", "b200")
    b = compute_stats(get_model("llama3_8b"), 16, "float8", "b200")
    assert b.fwd_us == pytest.approx(a.fwd_us / 2, rel=1e-9)
    assert b.forward_flops == a.forward_flops


def test_mi355x_preset_is_faster_than_b200():
    a = compute_stats(get_model("llama3_8b"), 16, "bfloat16", "b200")
    m = compute_stats(get_model("llama3_8b"), 16, "bfloat16", "mi355x")
    assert m.fwd_us == pytest.approx(a.fwd_us * 2.25 / 2.5, rel=1e-6)
    assert "MI355X" in m.device


def test_mixtral_analytic_non_expert_count():
    m = get_model("mixtral_8x7b")
    # embeddings (2 x 32000 x 4096) + 32 x (attention + router + norms) + final norm
    assert m.non_expert_params() == 1605636096
    assert m.total_params() == 46702792704


def test_aliases_and_unknown():
    assert get_model("llama3-8b") is MODELS["llama3_8b"]
    with pytest.raises(KeyError):
        get_model("gpt5")


def test_shipped_files_match_generator(root):
    for path in glob.glob(os.path.join(root, "model_stats", "*.txt")):
        st = load_stats(path)
        name, batch, dtype = os.path.basename(path)[:-4].rsplit("_", 2)
        gen = compute_stats(get_model(name), int(batch), dtype, "b200")
        assert parse_stats_text(gen.text()).fwd_us == st.fwd_us
        assert st.model_size == gen.model_size


REF = "/root/reference/model_stats"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not mounted")
def test_all_reference_tables_reproduced(root):
    files = sorted(glob.glob(os.path.join(REF, "*.txt")))
    assert len(files) == 72
    for f in files:
        ref = load_stats(f)
        ours = load_stats(os.path.join(root, "model_stats", os.path.basename(f)))
        for k in ("model_size", "non_expert_size", "batch", "experts", "seq_len", "hidden"):
            assert getattr(ref, k) == getattr(ours, k), (f, k)
        for k in ("forward_flops", "backward_flops", "fwd_us", "bwd_us", "ffn_fwd_us", "ffn_bwd_us"):
            assert getattr(ref, k) == pytest.approx(getattr(ours, k), rel=1e-12, abs=0.011), (f, k)


def test_models_json_schema(root):
    import json
    for name, m in MODELS.items():
        with open(os.path.join(root, "models", name + ".json")) as f:
            j = json.load(f)
        # the reference consumes only these two keys (cpp/utils.hpp:279-294)
        assert j.get("num_encoder_blocks", 0) + j.get("num_decoder_blocks", 0) == m.layers
        assert j["embed_dim"] == m.hidden and j["ff_dim"] == m.ffn
        if m.experts > 1:
            assert j["moe_params"] == {"num_experts": 8, "num_experts_per_tok": 2}
