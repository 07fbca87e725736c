import json
from dlnetbench_amd import engine
doc = engine.run_native("hybrid_3d_moe", "tiny_moe_8_bfloat16", 1, 2, 1, base_path="tests/data", warmup=1, runs=2,
                        compute="gemm", backend="rccl", quiet=True, graph=True)
print(json.dumps(doc["global"]["dlnb"]["lane_graphs"], indent=1))
doc = engine.run_native("fsdp", "llama3_8b_16_bfloat16", 32, 1, base_path=".", warmup=1, runs=2,
                        compute="gemm", backend="rccl", quiet=True, graph=True, time_scale=0.05)
print(json.dumps(doc["global"]["dlnb"]["lane_graphs"], indent=1))
