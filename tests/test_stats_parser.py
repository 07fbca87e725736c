"""Stats-file parsing: the three layouts, by key, in Python and in the native parser."""
import os

import pytest

from dlnetbench_amd import _native
from dlnetbench_amd.utils.stats import parse_stats_text

SHIPPED = """Forward_Flops:2111062325329920
Backward_Flops:4222124650659840
Model_Size:8030261248
Non_Expert_size:0
Average_Forward_Time (us):938249.92
Average_Backward_Time (us):1876499.84
Batch_size:16
FFN_Average_Forward_Time (us):437849.96
FFN_Average_Backward_Time (us):875699.93
Experts:1
Seq_len:8192
Embedded_dim:4096
Device:NVIDIA B200-192GB (Single)
Dtype:bfloat16
Bytes_per_element:2.0
"""

# python/model_stats.py layout: no Non_Expert_size, Model_Size = non-expert count
GENERATOR_MOE = """Forward_Flops:100
Backward_Flops:200
Model_Size:1605636096
Average_Forward_Time (us):10.5
Average_Backward_Time (us):21.0
Batch_size:4
FFN_Average_Forward_Time (us):5.0
FFN_Average_Backward_Time (us):10.0
Experts:8
Seq_len:32768
Embedded_dim:4096
Device:x
Dtype:bfloat16
Bytes_per_element:2.0
"""


def test_shipped_layout():
    st = parse_stats_text(SHIPPED)
    assert st.format == "shipped"
    assert st.model_size == 8030261248 and st.non_expert_size == 0
    assert st.fwd_us == 938249.92 and st.bwd_us == 1876499.84  # not truncated (reference #13)
    assert (st.batch, st.seq_len, st.hidden, st.experts) == (16, 8192, 4096, 1)


def test_generator_layout_is_not_misread():
    st = parse_stats_text(GENERATOR_MOE)
    assert st.format == "generator"
    assert st.batch == 4  # the reference's positional parser would read 21.0 here
    assert st.non_expert_size == 1605636096
    assert st.experts == 8


def test_lowercase_key_variant():
    st = parse_stats_text(SHIPPED.replace("Non_Expert_size", "non_expert_size"))
    assert st.format == "shipped"


def test_missing_key_raises():
    with pytest.raises(ValueError):
        parse_stats_text("\n".join(SHIPPED.splitlines()[:6]))


def test_native_parser_agrees(tmp_path):
    for text in (SHIPPED, GENERATOR_MOE):
        p = tmp_path / "m.txt"
        p.write_text(text)
        nat = _native.parse_stats(str(p))
        py = parse_stats_text(text)
        assert nat["model_size"] == py.model_size
        assert nat["non_expert_size"] == py.non_expert_size
        assert nat["batch_size"] == py.batch
        assert nat["avg_forward_time_us"] == pytest.approx(py.fwd_us)
        assert nat["format"] == py.format


def test_native_parser_errors(tmp_path):
    with pytest.raises(_native.NativeError):
        _native.parse_stats(str(tmp_path / "missing.txt"))
    p = tmp_path / "bad.txt"
    p.write_text("Forward_Flops:1\nno colon here\n")
    with pytest.raises(_native.NativeError):
        _native.parse_stats(str(p))


def test_every_shipped_file_parses(root):
    for d in ("model_stats", "model_stats_mi355x"):
        for f in sorted(os.listdir(os.path.join(root, d))):
            nat = _native.parse_stats(os.path.join(root, d, f))
            assert nat["format"] == "dlnb" and nat["model_size"] > 0


def test_host_conversions_roundtrip():
    L = _native.lib()
    for v in (0.0, 1.0, -2.5, 3.140625, 448.0, 1e-3):
        assert L.dlnb_bf16_to_float(L.dlnb_float_to_bf16(v)) == pytest.approx(v, rel=1e-2, abs=1e-6)
    # OCP e4m3fn: max finite 448, saturating
    assert L.dlnb_fp8e4m3_to_float(L.dlnb_float_to_fp8e4m3(1000.0)) == 448.0
    assert L.dlnb_fp8e4m3_to_float(L.dlnb_float_to_fp8e4m3(-0.5)) == -0.5
    assert L.dlnb_fp8e4m3_to_float(0x7E) == 448.0


@pytest.mark.parametrize("M,N,cus,nf", [
    (8192, 1280, 256, 5),    # ViT-H / GPT-2-L FFN down (C5 stand-in): 160 square tiles -> 256 of 256 x 160
    (8192, 1024, 256, 4),    # ViT-L: 128 -> 256 of 256 x 128
    (8192, 1536, 256, 6),    # 192 -> 256 of 256 x 192
    (4096, 4096, 256, 8),    # 256 square tiles already fill the chip
    (8192, 4096, 256, 8),    # more tiles than CUs: the streaming square kernel
    (6144, 2048, 256, 8),    # 192 tiles; 256 x 128 would need two rounds (384), no 160 / 192 fit: square
    (8192, 1280, 224, 8),    # 224 CUs: 256 narrow tiles need 2 rounds of 5 > 1 round of 8
    (512, 768, 256, 3),      # 6 square tiles: 16 of 256 x 96 (3 units each) beat 12 of 256 x 128 (4)
    (8192, 768, 256, 3),     # ViT-B: 96 -> 256 of 256 x 96
    (8192, 1792, 256, 7),    # GPT-2-XL hidden (1600, stand-in 1792): 224 -> 256 of 256 x 224
    (8192, 5120, 256, 5),    # 640 square tiles = 2.5 rounds (cost 24); 1024 of 256 x 160 = 4 rounds (20)
    (8192, 3072, 256, 6),    # 384 = 1.5 rounds (16); 512 of 256 x 192 = 2 rounds (12)
    (8192, 6144, 256, 8),    # 768 = 3 rounds (24); 1024 of 256 x 192 = 4 (24): no saving
    (16384, 5120, 256, 8),   # 1280 = 5 rounds; 2048 of 256 x 160 = 8 rounds of 5: a tie
])
def test_fp8_narrow_tile_choice(M, N, cus, nf):
    """The one-shot MX fp8 kernel's tile width (gemm_tn_4wave_fp8 -> gemm_4wave_fp8_narrow_nf): the fewest rounds
    of tile work per CU. Host code only, runs without a GPU."""
    assert _native.lib().dlnb_gemm_narrow_nf(M, N, cus) == nf


def test_fp8_narrow_tile_choice_gpu_cases():
    """The tile widths test_gpu_kernels.py::test_gemm_fp8_narrow_tiles expects on a 256-CU MI355X."""
    L = _native.lib()
    for M, N, nf in [(2048, 1280, 4), (8192, 1280, 5), (7168, 1280, 5), (8192, 1536, 6), (8192, 1024, 4),
                     (768, 512, 4), (6144, 2048, 8), (8192, 768, 3), (512, 768, 3)]:
        assert L.dlnb_gemm_narrow_nf(M, N, 256) == nf, (M, N)
