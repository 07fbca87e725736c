"""Tooling: sweep checkpoint/resume, report parsing to DataFrames, plots,
fault injection / failure detection, CLI contract of the binaries."""
import json
import os
import subprocess

import pytest

from dlnetbench_amd.tools import plots, sweep
from dlnetbench_amd.utils import launch, report


@pytest.fixture(scope="module")
def bindir(root):
    d = os.path.join(root, "build", "bin")
    if not os.path.exists(os.path.join(d, "dp")):
        pytest.skip("binaries not built")
    return d


def test_sweep_runs_and_resumes(tmp_path, bindir):
    out = tmp_path / "r.jsonl"
    assert sweep.main(["--quick", "--out", str(out), "--bin", bindir]) == 0
    lines = out.read_text().splitlines()
    assert len(lines) == 4
    recs = [json.loads(l) for l in lines]
    assert all(r["exit_code"] == 0 and r["summary"]["median_ms"] > 0 for r in recs)
    # resume: nothing left to do
    assert sweep.main(["--quick", "--out", str(out), "--bin", bindir]) == 0
    assert len(out.read_text().splitlines()) == 4
    # partial file -> only the missing points run again
    out.write_text("\n".join(lines[:2]) + "\n")
    assert sweep.main(["--quick", "--out", str(out), "--bin", bindir]) == 0
    keys = [json.loads(l)["key"] for l in out.read_text().splitlines()]
    assert len(keys) == 4 and len(set(keys)) == 4


def test_sweep_expansion_env_matrix():
    spec = {"points": [{"strategy": "fsdp", "model": "m", "params": [4, "W"], "world": [2, 4],
                        "env": {"NCCL_PROTO": ["Simple", "LL128"], "NCCL_ALGO": "Ring"}}]}
    pts = list(sweep.expand(spec))
    assert len(pts) == 4
    assert {tuple(p["params"]) for p in pts} == {(4, 2), (4, 4)}
    assert len({sweep.point_key(p) for p in pts}) == 4


def test_report_dataframes(tmp_path, bindir, data_dir):
    code, outs = launch.launch(2, [os.path.join(bindir, "fsdp"), "tiny_dense_8_bfloat16", "4", "2", data_dir,
                                   "--quiet", "-w", "1", "-r", "2"], timeout=60, capture=True)
    assert code == 0
    doc = report.parse_output(outs[0])["fsdp"]
    assert report.validate(doc, expected_world=2, nodes=1) == []
    assert report.validate(doc, expected_world=4) != []
    rt, comm = report.fsdp_dataframes(doc)
    assert len(rt) == 2 * 2 and len(comm) == 2 * 2 * 4
    assert set(["runtime", "allgather", "barrier", "rank"]) <= set(rt.columns)
    assert set(["allgather_wait_fwd", "allgather_wait_bwd", "reduce_scatter", "unit_idx"]) <= set(comm.columns)
    code, outs = launch.launch(2, [os.path.join(bindir, "dp"), "tiny_dense_8_bfloat16", "3", data_dir, "--quiet",
                                   "-w", "0", "-r", "3"], timeout=60, capture=True, env=dict(os.environ, NCCL_PROTO="Simple"))
    doc = report.parse_output(outs[0])["dp"]
    df = report.dp_dataframe(doc)
    assert len(df) == 6 and (df["protocol"] == "Simple").all()
    assert {"runtime", "barrier_time", "energy_consumed", "msg_size_avg_bytes"} <= set(df.columns)
    s = report.summary(doc)
    assert s["busbw_GBps"]["allreduce"] > 0
    # extensions: context parallel and 4-D sections
    code, outs = launch.launch(4, [os.path.join(bindir, "hybrid_cp"), "tiny_dense_8_bfloat16", "2", data_dir, "--quiet",
                                   "-w", "0", "-r", "2"], timeout=60, capture=True)
    assert code == 0
    df = report.cp_dataframe(report.parse_output(outs[0])["dp_cp"])
    assert len(df) == 4 * 2 and {"cp_comm_time", "cp_exposed_time", "dp_exposed_time", "cp_id"} <= set(df.columns)
    code, outs = launch.launch(4, [os.path.join(bindir, "hybrid_4d"), "tiny_moe_8_bfloat16", "1", "2", "2", "2",
                                   data_dir, "--quiet", "-w", "0", "-r", "2"], timeout=60, capture=True)
    assert code == 0
    df = report.hybrid_dataframe(report.parse_output(outs[0])["dp_pp_tp_ep"])
    assert len(df) == 4 * 2 and {"tp_comm_time", "ep_comm_time"} <= set(df.columns)
    code, outs = launch.launch(4, [os.path.join(bindir, "hybrid_2d"), "tiny_deep_8_bfloat16", "4", "8", data_dir,
                                   "--quiet", "-w", "0", "-r", "2", "--pp-schedule", "dualpipe"], timeout=60, capture=True)
    assert code == 0
    df = report.hybrid_dataframe(report.parse_output(outs[0])["dp_pp"])
    assert len(df) == 4 * 2 and (df["pp_schedule"] == "dualpipe").all() and "pp_mirror_time" in df.columns


def test_plots(tmp_path, bindir):
    out = tmp_path / "r.jsonl"
    sweep.main(["--quick", "--out", str(out), "--bin", bindir])
    for kind in ("scaling", "barrier", "pareto"):
        png = tmp_path / f"{kind}.png"
        assert plots.main([kind, str(out), "-o", str(png)]) == 0
        assert png.exists() and png.stat().st_size > 1000


def test_knob_plots(tmp_path, bindir, data_dir):
    """Protocol x algorithm facets with threads x channels series, and the per-model energy Pareto
    (plot_dp.py:23-26, plots_pareto_energy.py:107-234): a real 2-point knob sweep on the CPU backend,
    then synthetic copies filling a 2 x 2 x 2 knob grid with known values."""
    import copy
    spec = {"base_path": data_dir, "points": [
        {"strategy": "dp", "model": "tiny_dense_8_bfloat16", "params": [2], "world": [2],
         "opts": {"warmup": 0, "runs": 2, "backend": "cpu"},
         "env": {"NCCL_PROTO": ["Simple", "LL128"], "NCCL_ALGO": "Ring"}}]}
    sf = tmp_path / "spec.json"
    sf.write_text(json.dumps(spec))
    out = tmp_path / "r.jsonl"
    assert sweep.main([str(sf), "--out", str(out), "--bin", bindir]) == 0
    recs = plots.load_records(str(out))
    assert [plots.knobs(r)["protocol"] for r in recs] == ["Simple", "LL128"]
    assert plots.knobs(recs[0]) == {"protocol": "Simple", "algorithm": "Ring", "threads": "default",
                                    "channels": "default"}
    grid = []
    for proto in ("Simple", "LL128"):
        for algo in ("Ring", "Tree"):
            for nt in ("256", "512"):
                for w in (2, 4):
                    r = copy.deepcopy(recs[0])
                    r["point"]["env"] = {"NCCL_PROTO": proto, "NCCL_ALGO": algo, "NCCL_NTHREADS": nt,
                                         "NCCL_MAX_NCHANNELS": "8"}
                    r["report"]["global"]["world_size"] = w
                    r["report"]["global"]["dlnb"]["iteration"]["median_ms"] = 10.0 + w + (nt == "512")
                    for rk in r["report"]["ranks"]:
                        rk["energy_consumed"] = [5.0 + (algo == "Tree")] * 2
                    grid.append(r)
    gf = tmp_path / "grid.jsonl"
    gf.write_text("\n".join(json.dumps(r) for r in grid) + "\n")
    counts = plots.plot_knobs(grid, str(tmp_path / "k.png"))
    assert counts == {(p, a): 4 for p in ("LL128", "Simple") for a in ("Ring", "Tree")}
    assert plots.plot_knobs(grid, str(tmp_path / "kb.png"), metric="barrier")[("Simple", "Ring")] == 4
    assert plots.plot_knobs_pareto(grid, str(tmp_path / "p.png")) == {"tiny_dense_8_bfloat16": 16}
    for kind, extra in (("knobs", []), ("knobs", ["--metric", "barrier"]), ("knobs-pareto", [])):
        png = tmp_path / f"cli_{kind}.png"
        assert plots.main([kind, str(gf), "-o", str(png), *extra]) == 0 and png.stat().st_size > 1000


def test_zoom_inset_and_style_maps(tmp_path):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots()
    ax.plot([1, 2, 3, 4], [10, 1, 1.1, 1.2], marker="o")
    ax.scatter([2.5], [1.05])
    ins = plots.add_zoom_inset(ax, (1.8, 4.2, 0.9, 1.3))
    assert ins.get_xlim() == (1.8, 4.2) and ins.get_ylim() == (0.9, 1.3)
    assert len(ins.get_lines()) == 1 and len(ins.collections) == 1
    assert len(ax.patches) == 1  # the dashed zoom rectangle
    fig.savefig(tmp_path / "z.png")
    cm = plots.create_color_map(range(12))
    assert cm[0] == cm[10] != cm[1]
    assert plots.create_marker_map(["a", "b"]) == {"a": "o", "b": "s"}
    assert plots.create_linestyle_map(range(5))[4] == "-"
    assert plots.pareto_staircase([(1, 5), (2, 3), (4, 1), (3, 4)]) == [(1, 5), (2, 5), (2, 3), (4, 3), (4, 1)]


def test_plot_utils():
    assert plots.format_bytes(1536) == "1.5 KiB"
    assert plots.format_bytes(512) == "512 B"
    assert plots.parse_bytes("1.5 KiB") == 1536
    assert plots.parse_bytes("2GB") == 2_000_000_000
    pts = [(1, 5), (2, 3), (3, 4), (4, 1), (2.5, 2.9)]
    assert plots.pareto_front(pts) == [0, 1, 4, 3]


@pytest.mark.parametrize("mode,code", [("exit", 42), ("throw", 2), ("hang", 17)])
def test_fault_injection_is_detected(mode, code, bindir, data_dir):
    env = dict(os.environ, DLNB_INJECT_FAULT=f"rank=1,iter=1,mode={mode}", DLNB_TIMEOUT="5")
    rc, outs = launch.launch(2, [os.path.join(bindir, "dp"), "tiny_dense_8_bfloat16", "2", data_dir, "--quiet",
                                 "-w", "2", "-r", "2"], timeout=90, capture=True, env=env)
    text = "".join(o or "" for o in outs)
    assert rc == code, text[-2000:]
    assert "DLNB_INJECT_FAULT" in text


def test_cli_contract(bindir, data_dir):
    r = subprocess.run([os.path.join(bindir, "dp"), "-h"], capture_output=True, text=True)
    assert r.returncode == 0 and "<model> <num_buckets> <base_path>" in r.stdout
    r = subprocess.run([os.path.join(bindir, "hybrid_3d"), "-h"], capture_output=True, text=True)
    assert "<num_tensor_shards>" in r.stdout and "default 3" in r.stdout
    r = subprocess.run([os.path.join(bindir, "fsdp"), "m", "4"], capture_output=True, text=True)
    assert r.returncode == 1 and "expected 4 positional" in r.stderr
    r = subprocess.run([os.path.join(bindir, "dp"), "m", "x", "."], capture_output=True, text=True)
    assert r.returncode == 1 and "invalid integer" in r.stderr
    r = subprocess.run([os.path.join(bindir, "dp"), "nope_1_bfloat16", "2", data_dir, "--quiet"],
                       capture_output=True, text=True)
    assert r.returncode == 2 and "does not exist" in r.stderr
    r = subprocess.run([os.path.join(bindir, "dlnb"), "fsdp", "-h"], capture_output=True, text=True)
    assert r.returncode == 0 and "<sharding_factor>" in r.stdout


def test_topology_print(bindir, data_dir):
    code, outs = launch.launch(2, [os.path.join(bindir, "dp"), "tiny_dense_8_bfloat16", "2", data_dir, "-w", "0",
                                   "-r", "1"], timeout=60, capture=True)
    assert code == 0
    assert "=== topology: 2 ranks on 1 node(s) ===" in outs[0]
    env = dict(os.environ, SLURM_TOPOLOGY_ADDR="root.sw1.nodeA")
    code, outs = launch.launch(2, [os.path.join(bindir, "dp"), "tiny_dense_8_bfloat16", "2", data_dir, "-w", "0",
                                   "-r", "1"], timeout=60, capture=True, env=env)
    assert "sw1" in outs[0] and "ranks [0,1]" in outs[0]


def test_plan_cli(capsys, root):
    from dlnetbench_amd.parallel import plan
    assert plan.main(["hybrid_3d", "llama3_70b_16_bfloat16", "2", "4", "4", "--world", "8", "--base", root]) == 0
    d = json.loads(capsys.readouterr().out)
    assert d["params"]["num_tensor_shards"] == 4


@pytest.mark.parametrize("prog,args,extra", [("fsdp", ["tiny_dense_8_bfloat16", "4", "2"], ["--timeline", "{tmp}"]),
                                             ("hybrid_3d_moe", ["tiny_moe_8_bfloat16", "2", "2", "1"], []),
                                             ("hybrid_3d", ["tiny_dense_8_bfloat16", "2", "2", "1"], [])])
def test_asan_build_is_clean(prog, args, extra, asan_bindir, data_dir, tmp_path):
    """Host AddressSanitizer build (make asan, built on demand): no memory errors in the runtime (the fsdp
    case: zero-copy shared-memory collectives on registered buffers, with the device timeline on)."""
    b = os.path.join(asan_bindir, prog)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    extra = [x.replace("{tmp}", str(tmp_path / "tl.json")) for x in extra]
    code, outs = launch.launch(2, [b, *args, data_dir, "--quiet", "-w", "1", "-r", "2", *extra], timeout=120,
                               capture=True, env=env)
    text = "".join(o or "" for o in outs)
    assert code == 0 and "AddressSanitizer" not in text, text[-3000:]


@pytest.mark.parametrize("prog,args,extra", [("fsdp", ["tiny_dense_8_bfloat16", "4", "4"], []),
                                             ("hybrid_2d", ["tiny_deep_8_bfloat16", "4", "8"],
                                              ["--pp-schedule", "interleaved"]),
                                             ("hybrid_3d_moe", ["tiny_moe_8_bfloat16", "2", "4", "2"],
                                              ["--ep-overlap", "--timeline", "/dev/null"])])
def test_tsan_loopback_threads_race_free(prog, args, extra, tsan_bindir, data_dir):
    """Host ThreadSanitizer build (make tsan, built on demand): 8 loopback rank threads on the CPU device,
    no data races."""
    b = os.path.join(tsan_bindir, prog)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "DLNB_RANK", "DLNB_WORLD_SIZE")}
    env["TSAN_OPTIONS"] = "halt_on_error=1"
    p = subprocess.run([b, *args, data_dir, *extra, "--backend", "loopback-cpu", "--ranks", "8", "--quiet",
                        "-w", "1", "-r", "2"], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0 and "ThreadSanitizer" not in p.stderr, p.stderr[-3000:]


def test_graph_needs_gpu(bindir, data_dir):
    p = subprocess.run([os.path.join(bindir, "dp"), "tiny_dense_8_bfloat16", "2", data_dir, "--backend",
                        "cpu", "--graph", "-w", "0", "-r", "1"], capture_output=True, text=True)
    assert p.returncode == 2 and "graph" in p.stderr


def test_unified_cli(tmp_path, data_dir, root):
    from dlnetbench_amd.__main__ import main
    out = tmp_path / "r.json"
    assert main(["run", "-n", "2", "dp", "tiny_dense_8_bfloat16", "2", data_dir, "--backend", "cpu", "-w", "0", "-r",
                 "1", "--silent", "--json", str(out)]) == 0
    assert json.loads(out.read_text())["global"]["world_size"] == 2
    assert main(["run", "bogus"]) == 1
    assert main(["nope"]) == 1
    assert main(["plan", "fsdp", "llama3_8b_16_bfloat16", "32", "8", "--world", "8", "--base", root]) == 0


def test_prof_merge_folds_counters_into_report(tmp_path):
    """tools/prof_merge.py: rocprofv3 kernel trace + PMC CSVs -> global.dlnb.counters per kernel class."""
    from dlnetbench_amd.tools import prof_merge
    tr = tmp_path / "prof" / "host" / "123"
    tr.mkdir(parents=True)
    rows = [("void dlnb::kernels::gemm_8phase_kernel<false, true, false>(...)", 0, 2_000_000),
            ("void dlnb::kernels::gemm_8phase_kernel<false, true, false>(...)", 3_000_000, 5_000_000),
            ("ncclDevKernel_Generic_1(ncclDevKernelArgsStorage<4096ul>)", 100, 600_100),
            ("__amd_rocclr_copyBuffer", 0, 1000),
            ("void dlnb::xgmi::(anonymous namespace)::ar2_kernel<(dlnb::DType)0>(...)", 0, 50_000)]
    with open(tr / "x_kernel_trace.csv", "w") as f:
        f.write("Kind,Agent_Id,Kernel_Name,Start_Timestamp,End_Timestamp\n")
        for n, s, e in rows:
            f.write(f'KERNEL_DISPATCH,1,"{n}",{s},{e}\n')
    pm = tmp_path / "pmc"
    pm.mkdir()
    with open(pm / "y_counter_collection.csv", "w") as f:
        f.write("Dispatch_Id,Agent_Id,Kernel_Name,Counter_Name,Counter_Value,Start_Timestamp,End_Timestamp\n")
        g = "void dlnb::kernels::gemm_8phase_kernel<false, true, false>(...)"
        # 1 ms dispatch at 2 GHz: GUI = 2e6 cycles x 8 XCDs; MFMA busy half of 256 CUs x 4 SIMDs
        f.write(f'1,1,"{g}",GRBM_GUI_ACTIVE,16000000,0,1000000\n')
        f.write(f'1,1,"{g}",SQ_VALU_MFMA_BUSY_CYCLES,{0.5 * 2e6 * 1024},0,1000000\n')
        f.write(f'1,1,"{g}",SQ_INSTS_VALU_MFMA_MOPS_BF16,{1e15 * 1e-3 / 512},0,1000000\n')
        f.write(f'1,1,"{g}",FETCH_SIZE,{4e9 / 1024},0,1000000\n')
    pm2 = tmp_path / "pmc2"  # a second pass (WRITE_SIZE did not fit the first): 2 ms dispatch
    pm2.mkdir()
    with open(pm2 / "z_counter_collection.csv", "w") as f:
        f.write("Dispatch_Id,Agent_Id,Kernel_Name,Counter_Name,Counter_Value,Start_Timestamp,End_Timestamp\n")
        f.write(f'1,1,"{g}",WRITE_SIZE,{2e9 / 1024},0,2000000\n')
    rep_path = tmp_path / "r.json"
    rep_path.write_text(json.dumps({"section": "fsdp", "global": {"dlnb": {"iteration": {}}}, "ranks": []}))
    assert prof_merge.main([str(rep_path), str(tmp_path / "prof"), str(pm), str(pm2)]) == 0
    c = json.loads(rep_path.read_text())["global"]["dlnb"]["counters"]
    cl = c["classes"]
    assert cl["compute_gemm"]["calls"] == 2 and cl["compute_gemm"]["time_ms"] == pytest.approx(4.0)
    assert cl["rccl"]["calls"] == 1 and cl["copy"]["calls"] == 1 and cl["xgmi"]["calls"] == 1
    assert cl["compute_gemm"]["clock_GHz"] == pytest.approx(2.0)
    assert cl["compute_gemm"]["mfma_busy"] == pytest.approx(0.5)
    assert cl["compute_gemm"]["mfma_TFLOPs"] == pytest.approx(1000.0, rel=1e-3)
    assert cl["compute_gemm"]["fabric_GBps"] == pytest.approx(5000.0, rel=1e-3)
    assert c["total_kernel_ms"] == pytest.approx(4.0 + 0.6 + 0.001 + 0.05)
    assert sum(v["time_pct"] for v in cl.values()) == pytest.approx(100.0, abs=0.05)


def test_xgmi_kernels_fit_the_cu_budget(root):
    """Every peer-waiting xgmi kernel fits 4 blocks of 512 threads per CU on
    registers (<= 64 per lane, no scratch), which the comm-lane CU budget
    (comm_xgmi.cpp, runner.cpp) assumes; read from the gfx950 code object."""
    from dlnetbench_amd.tools.kernel_resources import kernel_resources
    ks = kernel_resources(os.path.join(root, "csrc", "kernels", "xgmi.hip"))
    peer = [k for k in ks if "local_" not in k["name"]]
    assert len(peer) == 31, [k["name"] for k in peer]
    for k in peer:
        assert k["max_threads"] == 512, k
        assert k["waves_per_simd"] == 8 and k["blocks_per_cu_regs"] >= 4, k
        assert k["scratch"] == 0, k


def test_prof_merge_clock_from_long_dispatches_only(tmp_path):
    """GRBM_GUI_ACTIVE over a short dispatch includes the collection window's
    setup cycles: a 10-us copy kernel must not report a 5 GHz clock. Classes
    without long dispatches take the job's clock; an impossible clock raises."""
    from dlnetbench_amd.tools import prof_merge
    pm = tmp_path / "pmc"
    pm.mkdir()
    g = "void dlnb::kernels::gemm_8phase_kernel<false, true, false>(...)"
    cp = "__amd_rocclr_copyBuffer"
    with open(pm / "y_counter_collection.csv", "w") as f:
        f.write("Dispatch_Id,Agent_Id,Kernel_Name,Counter_Name,Counter_Value,Start_Timestamp,End_Timestamp\n")
        # two long GEMM dispatches at 2.0 GHz (2 ms, 3 ms)
        for d, ms in ((1, 2.0), (2, 3.0)):
            f.write(f'{d},1,"{g}",GRBM_GUI_ACTIVE,{8 * 2.0e9 * ms * 1e-3},0,{int(ms * 1e6)}\n')
            f.write(f'{d},1,"{g}",SQ_VALU_MFMA_BUSY_CYCLES,{0.6 * 2.0e9 * ms * 1e-3 * 1024},0,{int(ms * 1e6)}\n')
        # 50 short copies of 10 us, each with 30k cycles of window overhead (naive clock: 5 GHz)
        for d in range(3, 53):
            f.write(f'{d},1,"{cp}",GRBM_GUI_ACTIVE,{8 * (2.0e9 * 10e-6 + 30000)},0,10000\n')
    rep = prof_merge.merge({}, [str(pm)])
    cl = rep["global"]["dlnb"]["counters"]["classes"]
    assert cl["compute_gemm"]["clock_GHz"] == pytest.approx(2.0) and cl["compute_gemm"]["clock_source"] == "class"
    assert cl["compute_gemm"]["mfma_busy"] == pytest.approx(0.6)
    assert cl["copy"]["clock_GHz"] == pytest.approx(2.0) and cl["copy"]["clock_source"] == "job"
    for c in cl.values():
        assert c.get("clock_GHz", 0) <= 2.4
    # a long dispatch whose GUI count implies 3 GHz is rejected, not reported
    with open(pm / "y_counter_collection.csv", "a") as f:
        f.write(f'99,1,"{g}",GRBM_GUI_ACTIVE,{8 * 3.0e9 * 10 * 1e-3 * 10},0,10000000\n')
    with pytest.raises(ValueError, match="GHz"):
        prof_merge.merge({}, [str(pm)])


def test_prof_merge_busy_on_the_deadline_grid(tmp_path):
    """The deadline GEMM occupies deadline_grid CUs (224 of 256): its MFMA busy
    fraction on those CUs is reported next to the whole-chip one."""
    from dlnetbench_amd.tools import prof_merge
    pm = tmp_path / "pmc"
    pm.mkdir()
    g = "void dlnb::kernels::gemm_8phase_kernel<false, true, true>(...)"
    with open(pm / "y_counter_collection.csv", "w") as f:
        f.write("Dispatch_Id,Agent_Id,Kernel_Name,Counter_Name,Counter_Value,Start_Timestamp,End_Timestamp\n")
        f.write(f'1,1,"{g}",GRBM_GUI_ACTIVE,{8 * 2.0e9 * 1e-3},0,1000000\n')
        f.write(f'1,1,"{g}",SQ_VALU_MFMA_BUSY_CYCLES,{0.7 * 2.0e9 * 1e-3 * 224 * 4},0,1000000\n')
    rep = {"global": {"dlnb": {"compute": {"deadline_grid": 224}}}}
    c = prof_merge.merge(rep, [str(pm)])["global"]["dlnb"]["counters"]["classes"]["compute_gemm"]
    assert c["mfma_busy"] == pytest.approx(0.7 * 224 / 256) and c["mfma_busy_on_grid"] == pytest.approx(0.7)
    assert c["grid_cus"] == 224


def test_slurm_environment_bootstrap(tmp_path, data_dir, root):
    """Rank identity from Slurm's variables (SLURM_PROCID / SLURM_NTASKS /
    SLURM_LOCALID, what srun in scripts/slurm/dlnb.sbatch provides) with the
    store on DLNB_STORE_ADDR: 2 processes rendezvous and run DP on the CPU
    backend."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    out = tmp_path / "r.json"
    procs = []
    for r in range(2):
        env = {k: v for k, v in os.environ.items() if not k.startswith(("DLNB_", "RANK", "WORLD_SIZE", "LOCAL_"))}
        env.update({"SLURM_PROCID": str(r), "SLURM_NTASKS": "2", "SLURM_LOCALID": str(r),
                    "DLNB_STORE_ADDR": f"127.0.0.1:{port}", "SLURM_TOPOLOGY_ADDR": "root.sw0.node0"})
        args = [os.path.join(root, "build", "bin", "dp"), "tiny_dense_8_bfloat16", "4", data_dir, "--backend", "cpu",
                "--compute", "sleep", "-w", "1", "-r", "2", "--quiet"] + (["--json", str(out)] if r == 0 else [])
        procs.append(subprocess.Popen(args, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), res[0][1][-1500:] + res[1][1][-1500:]
    d = json.loads(out.read_text())
    assert d["global"]["world_size"] == 2 and sorted(r["rank"] for r in d["ranks"]) == [0, 1]
    assert [r["local_rank"] for r in sorted(d["ranks"], key=lambda r: r["rank"])] == [0, 1]



def test_every_env_knob_is_documented(root):
    """docs/KNOBS.md lists every DLNB_* variable the native runtime and the Python tools read."""
    import re
    pat = re.compile(r'(?:getenv|env_[a-z]+|environ\.get|environ\[)\(?\s*\{?"(DLNB_[A-Z0-9_]+)"')
    used = set()
    for top in ("csrc", "dlnetbench_amd"):
        for d, _, files in os.walk(os.path.join(root, top)):
            for f in files:
                if f.endswith((".cpp", ".hpp", ".hip", ".py")):
                    with open(os.path.join(d, f), errors="replace") as fh:
                        used |= set(pat.findall(fh.read()))
    with open(os.path.join(root, "bench.py")) as fh:
        used |= set(pat.findall(fh.read()))
    with open(os.path.join(root, "docs", "KNOBS.md")) as fh:
        doc = fh.read()
    assert len(used) > 30
    missing = sorted(k for k in used if f"`{k}`" not in doc)
    assert not missing, f"undocumented knobs: {missing}"
