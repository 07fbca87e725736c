"""Architecture registry for the nine benchmark models.

The reference's generator (python/model_stats.py:30-42, :101-145) downloads
each Hugging Face config *and the full weights* to count parameters. There
is no network here, and counting parameters does not need weights: every
model below is described by its HF config values and its parameter count is
derived analytically (embeddings, attention with GQA, gated/ungated MLP,
experts, norms, ViT patch/pos/pooler). The analytic counts reproduce the
``Model_Size`` values the reference ships in ``model_stats/*.txt``
exactly (checked in tests/test_models.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional


@dataclass(frozen=True)
class ModelArch:
    name: str                 # our file stem, e.g. "llama3_8b"
    hf_name: str              # Hugging Face id the values come from
    family: str               # "gpt2" | "llama" | "mixtral" | "vit"
    hidden: int
    layers: int
    heads: int
    ffn: int
    seq_len: int              # N used by the roofline (positions / patches+1)
    vocab: int = 0
    kv_heads: int = 0         # 0 = heads (no GQA)
    experts: int = 1
    top_k: int = 1
    tie_embeddings: bool = False
    image_size: int = 0
    patch_size: int = 0
    # Value written to Non_Expert_size when it differs from the analytic one
    # (the reference hand-edited Mixtral to a round 1.7e9,
    # model_stats/mixtral_8x7b_32_bfloat16.txt:3-4).
    non_expert_override: Optional[int] = None
    # Extra keys for models/<name>.json beyond the reference schema.
    json_extra: Dict[str, object] = field(default_factory=dict)

    @property
    def kv(self) -> int:
        return self.kv_heads or self.heads

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    # ---------------------------------------------------------- parameters
    def attention_params(self) -> int:
        d, hd = self.hidden, self.head_dim
        if self.family in ("gpt2", "vit"):
            return 3 * (d * d + d) + (d * d + d)  # qkv + out, with biases
        kvd = self.kv * hd
        return d * d + 2 * d * kvd + d * d       # q, k, v, o (no bias)

    def mlp_params_one_expert(self) -> int:
        d, f = self.hidden, self.ffn
        if self.family in ("gpt2", "vit"):
            return d * f + f + f * d + d           # fc + proj, with biases
        return 3 * d * f                           # gate, up, down

    def norm_params_per_layer(self) -> int:
        d = self.hidden
        if self.family in ("gpt2", "vit"):
            return 2 * 2 * d  # two LayerNorms with bias
        return 2 * d          # two RMSNorms

    def layer_params(self) -> int:
        p = self.attention_params() + self.norm_params_per_layer()
        p += self.experts * self.mlp_params_one_expert()
        if self.experts > 1:
            p += self.hidden * self.experts  # router
        return p

    def embedding_params(self) -> int:
        d = self.hidden
        if self.family == "vit":
            patch = 3 * self.patch_size * self.patch_size * d + d
            cls = d
            pos = self.seq_len * d
            return patch + cls + pos
        emb = self.vocab * d
        if self.family == "gpt2":
            emb += self.seq_len * d  # learned positions
        return emb

    def head_params(self) -> int:
        d = self.hidden
        if self.family == "vit":
            return 2 * d + (d * d + d)  # final LayerNorm + pooler
        final_norm = 2 * d if self.family == "gpt2" else d
        lm_head = 0 if self.tie_embeddings else self.vocab * d
        return final_norm + lm_head

    def total_params(self) -> int:
        return self.embedding_params() + self.layers * self.layer_params() + self.head_params()

    def expert_params(self) -> int:
        if self.experts <= 1:
            return 0
        return self.layers * self.experts * self.mlp_params_one_expert()

    def non_expert_params(self) -> int:
        return self.total_params() - self.expert_params()

    def stats_non_expert(self) -> int:
        """Value for the Non_Expert_size line: 0 for dense models (as shipped)."""
        if self.experts <= 1:
            return 0
        if self.non_expert_override is not None:
            return self.non_expert_override
        return self.non_expert_params()

    # ---------------------------------------------------------- models/*.json
    def arch_json(self) -> dict:
        """models/<name>.json: the reference schema (only the block counts are
        consumed, cpp/utils.hpp:279-294) plus the values used here."""
        j: dict = {
            "embed_dim": self.hidden,
            "num_heads": self.heads,
            "ff_dim": self.ffn,
            "seq_len": self.seq_len,
        }
        if self.family == "vit":
            j["num_encoder_blocks"] = self.layers
        else:
            j["num_encoder_blocks"] = 0
            j["num_decoder_blocks"] = self.layers
        if self.experts > 1:
            j["moe_params"] = {"num_experts": self.experts, "num_experts_per_tok": self.top_k}
        j["dlnb"] = {
            "hf_name": self.hf_name,
            "family": self.family,
            "vocab_size": self.vocab,
            "num_kv_heads": self.kv,
            "tie_word_embeddings": self.tie_embeddings,
            "image_size": self.image_size,
            "patch_size": self.patch_size,
            "total_params": self.total_params(),
            "non_expert_params": self.non_expert_params(),
        }
        j.update(self.json_extra)
        return j


def _vit(name, hf, d, L, H, ffn, patch, image=224):
    n = (image // patch) ** 2 + 1
    return ModelArch(name, hf, "vit", d, L, H, ffn, n, image_size=image, patch_size=patch)


MODELS: Dict[str, ModelArch] = {m.name: m for m in [
    _vit("vit_b", "google/vit-base-patch16-224", 768, 12, 12, 3072, 16),
    _vit("vit_l", "google/vit-large-patch16-224", 1024, 24, 16, 4096, 16),
    _vit("vit_h", "google/vit-huge-patch14-224-in21k", 1280, 32, 16, 5120, 14),
    ModelArch("gpt2_l", "gpt2-large", "gpt2", 1280, 36, 20, 5120, 1024, vocab=50257, tie_embeddings=True),
    ModelArch("gpt2_xl", "gpt2-xl", "gpt2", 1600, 48, 25, 6400, 1024, vocab=50257, tie_embeddings=True),
    ModelArch("minerva_7b", "sapienzanlp/Minerva-7B-instruct-v1.0", "llama", 4096, 32, 32, 14336, 4096,
              vocab=51264, kv_heads=8),
    ModelArch("llama3_8b", "meta-llama/Meta-Llama-3-8B", "llama", 4096, 32, 32, 14336, 8192,
              vocab=128256, kv_heads=8),
    ModelArch("llama3_70b", "meta-llama/Meta-Llama-3-70B", "llama", 8192, 80, 64, 28672, 8192,
              vocab=128256, kv_heads=8),
    ModelArch("mixtral_8x7b", "mistralai/Mixtral-8x7B-v0.1", "llama", 4096, 32, 32, 14336, 32768,
              vocab=32000, kv_heads=8, experts=8, top_k=2, non_expert_override=1_700_000_000),
]}

# Reference CLI names (python/model_stats.py:30-42 uses dashes).
ALIASES = {k.replace("_", "-"): k for k in MODELS}


def get_model(name: str) -> ModelArch:
    key = ALIASES.get(name, name)
    if key not in MODELS:
        raise KeyError(f"unknown model {name!r}; known: {sorted(MODELS)}")
    return MODELS[key]
