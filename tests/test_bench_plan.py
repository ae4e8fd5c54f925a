"""bench.py's multi-GPU planning and aggregation (CPU): `--gpus N` drives N
devices from one process (one host thread each), torch.distributed.run
launches one device per rank, and the whole-job rate is all devices' units
over the slowest device's time (independent streams, no
collective)."""
import importlib.util
import os
import threading

import pytest

from conftest import REPO


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_plan_threads_opens_every_device():
    b = _bench()
    p = b.plan_devices(8, {}, visible=8)
    assert p == {"mode": "threads", "rank": 0, "world": 1, "devices": list(range(8))}
    assert b.plan_devices(1, {}, visible=8)["devices"] == [0]
    with pytest.raises(SystemExit):
        b.plan_devices(4, {}, visible=2)  # never silently measure fewer GPUs than asked
    with pytest.raises(SystemExit):
        b.plan_devices(0, {}, visible=2)
    # rehearsal hook: two host threads on one device
    assert b.plan_devices(2, {"SDR_BENCH_DEVICES": "0,0"}, visible=1)["devices"] == [0, 0]
    with pytest.raises(SystemExit):
        b.plan_devices(3, {"SDR_BENCH_DEVICES": "0,0"}, visible=1)


def test_plan_ranks_one_device_each():
    b = _bench()
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    assert b.plan_devices(4, env, visible=8) == {"mode": "ranks", "rank": 2, "world": 4, "devices": [2]}
    with pytest.raises(SystemExit):
        b.plan_devices(8, env, visible=8)  # --gpus must match the launcher's world size


def test_plan_ranks_rehearsal_hook():
    """SDR_BENCH_DEVICES under torch.distributed.run: rank r runs device
    list[LOCAL_RANK], so two ranks can share the one GPU of a rehearsal box."""
    b = _bench()
    for r in (0, 1):
        env = {"WORLD_SIZE": "2", "RANK": str(r), "LOCAL_RANK": str(r), "SDR_BENCH_DEVICES": "0,0"}
        assert b.plan_devices(2, env, visible=1) == {"mode": "ranks", "rank": r, "world": 2, "devices": [0]}
    with pytest.raises(SystemExit):
        b.plan_devices(2, {"WORLD_SIZE": "2", "LOCAL_RANK": "1", "SDR_BENCH_DEVICES": "0"}, visible=1)
    with pytest.raises(SystemExit):
        b.plan_devices(2, {"WORLD_SIZE": "2", "LOCAL_RANK": "1"}, visible=1)  # no hook: device 1 is not there


def test_aggregate_is_all_units_over_the_slowest_device():
    b = _bench()
    units, steps = 1024 * 65540, 100
    agg = b.aggregate([10.0, 10.5, 9.8, 10.2], units, steps)
    assert agg["ms"] == 10.5
    assert agg["value"] == pytest.approx(4 * units * steps / 10.5e-3 / 1e6)
    assert agg["per_gpu_value"][2] == pytest.approx(units * steps / 9.8e-3 / 1e6)
    # weak scaling: N equal devices give N times one device
    one = b.aggregate([10.0], units, steps)["value"]
    assert b.aggregate([10.0] * 8, units, steps)["value"] == pytest.approx(8 * one)


def test_thread_driver_collects_every_device(monkeypatch):
    """main()'s thread mode with a fake per-device runner: every device is run
    in its own thread behind one barrier and reported."""
    b = _bench()
    seen = []
    lock = threading.Lock()

    def fake_run_device(cfg, device, seed, args, barrier=None, side=True):
        if barrier is not None:
            barrier()
        with lock:
            seen.append((device, threading.get_ident(), side))
        job = {"units": 1000, "bytes_per_pair": 8.4, "flops_per_unit": 41.4, "metric": "m", "bound": "hbm",
               "kind": "frontend_f32", "tolerance": None}
        return {"device": device, "ms": 1.0 + device, "wall": 0.01, "job": job}

    monkeypatch.setattr(b, "run_device", fake_run_device)

    class FakeCuda:
        @staticmethod
        def device_count():
            return 4

    class FakeTorch:
        cuda = FakeCuda

    import sys

    monkeypatch.setitem(sys.modules, "torch", FakeTorch)
    lines = []
    monkeypatch.setattr("builtins.print", lambda s, **k: lines.append(s))
    b.main(["--gpus", "4", "--steps", "10", "--no-cpu-baseline"])
    import json

    out = json.loads(lines[-1])
    assert sorted(d for d, _, _ in seen) == [0, 1, 2, 3]
    assert len({t for _, t, _ in seen}) == 4  # one host thread per device
    assert not any(side for _, _, side in seen)  # no side measurement at N > 1
    assert out["n_gpus"] == 4 and out["config"]["devices_opened"] == 4
    assert out["ms_per_step"] == pytest.approx(0.4)  # the slowest device: 4 ms / 10 steps
    assert len(out["per_gpu"]["value"]) == 4


def _rank_main(rank, world, port, q):
    """One torch.distributed.run rank of bench.main() with a fake device runner."""
    import importlib.util
    import io
    import json
    import os
    import sys

    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)

    def fake_run_device(cfg, device, seed, args, barrier=None, side=True):
        assert device == rank and not side
        barrier()  # the gloo barrier the real timed region uses
        job = {"units": 1000, "bytes_per_pair": 8.4, "flops_per_unit": 41.4, "metric": "m", "bound": "hbm",
               "kind": "frontend_f32", "tolerance": None}
        return {"device": device, "ms": 2.0 + rank, "wall": 0.01, "job": job}

    b.run_device = fake_run_device
    import torch

    torch.cuda.device_count = lambda: world
    out = io.StringIO()
    sys.stdout = out
    try:
        b.main(["--gpus", str(world), "--steps", "10", "--no-cpu-baseline"])
    finally:
        sys.stdout = sys.__stdout__
    text = out.getvalue().strip()
    q.put((rank, json.loads(text) if text else None))


def test_torchrun_ranks_use_gloo_and_max_time():
    """The torch.distributed.run path: each rank one device, the barrier and
    the max-over-ranks over a CPU gloo group (no device collective); rank 0
    alone prints, with the slowest rank's time."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[1] is None  # only rank 0 prints
    line = got[0]
    assert line["n_gpus"] == 2 and line["config"]["devices_opened"] == 2
    assert line["ms_per_step"] == pytest.approx(0.3)  # max(2, 3) ms / 10 steps
    assert line["per_gpu"]["ms_per_step"] == [pytest.approx(0.2), pytest.approx(0.3)]
    assert "gloo" in line["config"]["parallelism"]


def test_roofline_picks_the_binding_roof():
    """cfg2 (8.4 B, 41.3 FLOP per pair) is HBM-bound; the u8 wire format (2.4 B) and
    the resampler (4.735 B, 55.5 FLOP per input) sit above the exact-arithmetic ridge
    (one FLOP per lane per VALU issue: 78.65 TFLOP/s), so their line reports VALU."""
    b = _bench()
    base = {"metric": "m", "tolerance": None, "bound": "hbm"}
    cfg2 = dict(base, units=1024 * 65540, bytes_per_pair=8.4, flops_per_unit=41.3, kind="frontend_f32")
    r = b.roofline(cfg2, 0.1, "none")
    assert r["bound"] == "hbm" and r["frac"] == r["hbm_frac"]
    assert r["frac"] == pytest.approx(1024 * 65540 * 8.4 / 1e-4 / 1e9 / 8000, abs=1e-4)
    u8 = dict(cfg2, bytes_per_pair=2.4, kind="frontend_u8")
    r = b.roofline(u8, 0.08, "none")
    assert r["bound"] == "valu" and r["valu_peak_tflops"] == pytest.approx(157.3 / 2)
    assert b.roofline(u8, 0.08, "none", "fma")["valu_peak_tflops"] == pytest.approx(157.3)
    cfg3 = dict(base, units=1024 * 65600, bytes_per_pair=4.0 + 4.0 * 147 / 800,
                flops_per_unit=2.0 * 151 * 147 / 800, kind="resample")
    r = b.roofline(cfg3, 0.136, "none")
    assert r["bound"] == "valu" and r["frac"] == r["valu_frac"]
    assert r["hbm_frac"] == pytest.approx(0.29, abs=0.01)
    # the fp16 arm on the matrix cores: priced against the dense fp16 MFMA peak, bound "mfma"
    cfg5h = dict(base, units=2 * 1048576, bytes_per_pair=6.0, flops_per_unit=2.0 * 1024, kind="fir_block_f16",
                 f16_kernel="mfma")
    r = b.roofline(cfg5h, 0.0062, "none")
    assert r["bound"] == "mfma" and r["peak"] == pytest.approx(2500.0) and r["frac"] == r["valu_frac"]


@pytest.mark.parametrize("config", ["cfg2", "cfg3", "cfg5h", "mono0", "stereo0"])
def test_cpu_baseline_every_config(config):
    """bench.py attaches the reference CPU path to every config:
    the config's own kernel through oracle/cpu_bench (the reference's
    filter.cpp where it was built, else the C restatement), or the reference
    program for the program configs.  A tiny time budget here."""
    bench = _bench()

    exe_ref = os.path.join(REPO, "oracle", "_ref", "cpu_bench")
    if config in ("mono0", "stereo0") and not os.path.exists(os.path.join(REPO, "oracle", "_ref", "project_ref")):
        pytest.skip("the reference program is not built here")
    res = bench.cpu_baseline(0.4, config)
    assert res is not None and res["value"] > 0 and res["unit"] == "MS/s"
    assert res["kind"] == ("reference" if os.path.exists(exe_ref) else "port")
    assert res["cores"] >= 1 and res["value_1core"] > 0 and res["sample"]
    if config in ("mono0", "stereo0"):
        assert res["pcm_ok"]
    if config == "cfg2":
        assert "cfg1" in res or res["kind"] == "port"


@pytest.mark.parametrize("config", ["cfg2", "cfg2u8", "cfg3", "cfg4", "cfg4x8", "cfg5", "cfg5h", "mono0"])
def test_traffic_record_for_every_hbm_config(config):
    """Every config whose line prices HBM carries a PMC traffic record
    (profiles/traffic_<cfg>.json, FETCH_SIZE x2 + WRITE_SIZE per launch), and
    roofline() attaches it; against the closing record's algorithmic bytes it
    sits between 1x (every input fetched once) and the documented re-reads
    (cfg5's staged halo 1.52x, cfg5h's 1.19x, mono0's demod row 1.45x,
    DESIGN.md 5.1)."""
    import json

    b = _bench()
    with open(os.path.join(REPO, "profiles", f"traffic_{config}.json")) as f:
        t = json.load(f)["hbm_bytes_per_launch"]
    assert isinstance(t, int) and t > 0
    with open(os.path.join(REPO, "profiles", "r05ad", f"bench_{config}.json")) as f:
        alg = json.load(f)["roofline"]["algorithmic_bytes_per_launch"]
    assert 0.98 <= t / alg <= {"cfg5": 1.6, "mono0": 1.6, "cfg5h": 1.25}.get(config, 1.1)
    job = {"units": alg, "bytes_per_pair": 1.0, "flops_per_unit": 1.0, "kind": "frontend_f32"}
    assert b.roofline(job, 0.1, config)["traffic"] == t
