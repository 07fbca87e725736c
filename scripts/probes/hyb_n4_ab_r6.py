"""The bench's C3 / C4 rehearsal shapes (hybrid_3d tiny_deep 2 4 2, hybrid_3d_moe tiny_moe 2 8 2) as 4 ranks
sharing GPU 0 over the xgmi kernels, single graph (ranks share the device): the TP / EP placement and CTA A/B."""
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DATA = os.path.join(ROOT, "tests", "data")


def port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def run(binary, model, params, env_extra, W=4):
    p0, p1 = port(), port()
    tmp = tempfile.mkdtemp()
    procs = []
    for r in range(W):
        env = dict(os.environ, DLNB_NO_TORCH="1", DLNB_XGMI_TIMEOUT_S="60", RANK=str(r), WORLD_SIZE=str(W),
                   LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(W), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(p0),
                   DLNB_STORE_PORT=str(p1), **env_extra)
        cmd = [os.path.join(ROOT, "build", "bin", binary), model, *params, DATA, "--backend", "xgmi", "--devices",
               ",".join(["0"] * W), "--compute", "gemm", "--graph", "-w", "1", "-r", "3", "--quiet", "--silent",
               "--json", os.path.join(tmp, f"r{r}.json")]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    errs = []
    for p in procs:
        try:
            _, err = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            p.kill()
            _, err = p.communicate()
        errs.append((p.returncode, err[-300:]))
    if any(rc != 0 for rc, _ in errs):
        return {"error": errs}
    d = json.load(open(os.path.join(tmp, "r0.json")))
    g = d["global"]["dlnb"]
    r0 = [r for r in d["ranks"] if r.get("rank", 0) == 0][0]
    n = len(r0["runtimes"])
    return {"median_ms": round(g["iteration"]["median_ms"], 2), "per_run": [round(x * 1e3, 1) for x in r0["runtimes"]],
            **{k: round(sum(r0.get(k, [])) / n * 1e3, 2) for k in ("tp_comm_time", "tp_ar_time", "ep_comm_time", "ep_a2a_time", "pp_comm_time", "dp_comm_time")}}


which = sys.argv[1] if len(sys.argv) > 1 else "c3"
cfg = {"c3": ("hybrid_3d", "tiny_deep_8_bfloat16", ["2", "4", "2"]),
       "c4": ("hybrid_3d_moe", "tiny_moe_8_bfloat16", ["2", "8", "2"])}[which]
variants = {"default": {}, "ctas0": {"DLNB_INNER_CTAS": "0"}, "on_compute": {"DLNB_INNER_ON_COMPUTE": "1"},
            "on_compute_ctas0": {"DLNB_INNER_ON_COMPUTE": "1", "DLNB_INNER_CTAS": "0"}}
for name, env in variants.items():
    print(which, name, json.dumps(run(*cfg, env)), flush=True)
