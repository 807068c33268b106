"""Power, clocks and throttle state while the encode and the copy run sustained.

Back-to-back 1M x 1472 B encodes run ~0.517 ms, the streaming copy of the
same bytes ~0.471 ms, both at the same shader clock (GRBM_COUNT per ns).  This
runs each for a few seconds in turn while a thread samples the GPU's metrics
table (amdsmi, read-only) every 50 ms, and prints per phase the mean launch
time and the mean of every numeric metric that changes between phases
(power, gfx / memory / fabric clocks, temperatures, throttle bits).

usage: python tools/power_probe.py [--secs 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import threading
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def _flat(d, pre=""):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            out.update(_flat(v, f"{pre}{k}."))
        elif isinstance(v, (int, float)) and not isinstance(v, bool):
            out[pre + k] = float(v)
        elif isinstance(v, list) and v and all(isinstance(x, (int, float)) for x in v):
            vals = [float(x) for x in v if x not in (65535, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF)]
            if vals:
                out[pre + k + ".mean"] = sum(vals) / len(vals)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=3.0)
    args = ap.parse_args()
    import amdsmi
    amdsmi.amdsmi_init()
    handles = amdsmi.amdsmi_get_processor_handles()
    dev = torch.device("cuda", 0)
    lib = _native.tools_lib()
    lib.rudpx_copy_vpt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_void_p]
    L, M = 1472, 1 << 20
    tab, pay = batch.synth_batch(M, L, 0x5EED0004, device=dev)
    fr = torch.empty((M, L + 7), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    fns = {"encode": lambda: batch.pack_batch(tab, pay, 7, out=fr, want_csum=False),
           "copy": lambda: lib.rudpx_copy_vpt(pay.data_ptr(), fr.data_ptr(), M * L // 16, 1, 1, stream)}
    samples = []  # (phase, handle index, metrics)
    phase = {"name": "idle"}
    stop = threading.Event()

    def sampler():
        while not stop.is_set():
            for i, h in enumerate(handles):
                try:
                    m = _flat(amdsmi.amdsmi_get_gpu_metrics_info(h))
                except Exception as e:  # noqa: BLE001
                    m = {"error": str(e)}
                samples.append((phase["name"], i, m))
            time.sleep(0.05)
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    times = {}
    time.sleep(0.5)
    for name in ("encode", "copy", "encode", "copy"):
        key = name if name not in times else name + "_2"
        phase["name"] = key
        fn = fns[name]
        t_end = time.perf_counter() + args.secs
        ms = []
        while time.perf_counter() < t_end:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                fn()
            b.record()
            b.synchronize()
            ms.append(a.elapsed_time(b) / 20)
        times[key] = {"first_ms": ms[0], "mean_ms": sum(ms) / len(ms), "last_ms": ms[-1], "groups": len(ms)}
        phase["name"] = "idle"
        time.sleep(0.5)
    stop.set()
    th.join()
    # the GPU this process drove: the handle whose activity is highest while encoding
    act = {}
    for ph, i, m in samples:
        if ph.startswith("encode"):
            act.setdefault(i, []).append(m.get("average_gfx_activity", 0.0) + m.get("average_umc_activity", 0.0))
    gi = max(act, key=lambda i: sum(act[i]) / len(act[i])) if act else 0
    per = {}
    for ph, i, m in samples:
        if i == gi and "error" not in m:
            per.setdefault(ph, []).append(m)
    means = {ph: {k: sum(m.get(k, 0.0) for m in ms) / len(ms) for k in ms[0]} for ph, ms in per.items()}
    keys = [k for k in means.get("encode", {}) if len({round(means[p].get(k, 0.0), 3) for p in means}) > 1]
    print(json.dumps({"gpu_handle": gi, "launch_ms": times,
                      "metrics": {ph: {k: v[k] for k in keys if k in v} for ph, v in means.items()},
                      "samples": {ph: len(ms) for ph, ms in per.items()}}, indent=1))


if __name__ == "__main__":
    main()
