"""Model configuration cache (offline-first).

Reference: python/download_models.py pre-caches Hugging Face configs and
full weights for the stats generator (:21-36 registry, :42-76 download,
:83-119 CLI with --all / --config_only / --list). Weights are not needed
here: parameter counts are analytic (models/registry.py). This tool writes
HF-style ``config.json`` files for the registry models into a cache
directory, and only tries the Hugging Face hub when ``--hub`` is given and
``huggingface_hub`` plus a network are available.

    python -m dlnetbench_amd.tools.download_models --list
    python -m dlnetbench_amd.tools.download_models --all --config_only --cache ~/.cache/dlnb_models
"""
from __future__ import annotations

import argparse
import json
import os
import sys

from ..models.registry import MODELS, ModelArch, get_model


def hf_config(m: ModelArch) -> dict:
    if m.family == "vit":
        return {"model_type": "vit", "hidden_size": m.hidden, "num_hidden_layers": m.layers,
                "num_attention_heads": m.heads, "intermediate_size": m.ffn, "image_size": m.image_size,
                "patch_size": m.patch_size}
    if m.family == "gpt2":
        return {"model_type": "gpt2", "n_embd": m.hidden, "n_layer": m.layers, "n_head": m.heads,
                "n_positions": m.seq_len, "vocab_size": m.vocab}
    cfg = {"model_type": "mixtral" if m.experts > 1 else "llama", "hidden_size": m.hidden,
           "num_hidden_layers": m.layers, "num_attention_heads": m.heads, "num_key_value_heads": m.kv,
           "intermediate_size": m.ffn, "max_position_embeddings": m.seq_len, "vocab_size": m.vocab,
           "tie_word_embeddings": m.tie_embeddings}
    if m.experts > 1:
        cfg["num_local_experts"] = m.experts
        cfg["num_experts_per_tok"] = m.top_k
    return cfg


def write_config(m: ModelArch, cache: str) -> str:
    d = os.path.join(cache, m.hf_name.replace("/", "--"))
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, "config.json")
    with open(p, "w") as f:
        json.dump({**hf_config(m), "_name_or_path": m.hf_name, "_dlnb_total_params": m.total_params()}, f, indent=2)
    return p


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("models", nargs="*")
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--config_only", "--config-only", action="store_true", help="(always true offline)")
    ap.add_argument("--hub", action="store_true", help="also try snapshot_download from the HF hub")
    ap.add_argument("--cache", default=os.path.expanduser("~/.cache/dlnb_models"))
    a = ap.parse_args(argv)
    if a.list:
        for m in MODELS.values():
            print(f"{m.name:14s} {m.hf_name}")
        return 0
    names = list(MODELS) if a.all else a.models
    if not names:
        ap.error("give model names or --all")
    for n in names:
        m = get_model(n)
        print(write_config(m, a.cache))
        if a.hub:
            try:
                from huggingface_hub import snapshot_download
                snapshot_download(m.hf_name, allow_patterns=["config.json"] if a.config_only else None)
            except Exception as e:  # offline image: expected
                print(f"[download_models] hub download of {m.hf_name} unavailable: {e}", file=sys.stderr)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
