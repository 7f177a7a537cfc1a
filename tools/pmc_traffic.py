"""Turn the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/gpu_prof.sh into the per-launch HBM
traffic file bench.py reports as roofline.traffic (profiles/pmc_<workload>.json).

Units are calibrated on the 1 GiB device copy of tools/pmc_calib.py run under the same counters:
WRITE_SIZE reads in KiB exactly; FETCH_SIZE reads half of a wide streaming read (the gfx950
correction of MI355X_MICROARCH.md), so fetched bytes = FETCH_SIZE * 1024 * (2^30 / calib_bytes).
usage: python tools/pmc_traffic.py gpurun_out/prof WORKLOAD_DESCRIPTION > profiles/pmc_config3.json
"""
import json
import subprocess
import sys


def summary(path):
    return json.loads(subprocess.check_output(["python3", "tools/pmc_summary.py", path]))


def main():
    root, what = sys.argv[1], sys.argv[2]
    fetch, write = summary(f"{root}/fetch"), summary(f"{root}/write")
    cf = summary(f"{root}/cfetch")["__amd_rocclr_copyBuffer"]["FETCH_SIZE"]
    cw = summary(f"{root}/cwrite")["__amd_rocclr_copyBuffer"]["WRITE_SIZE"]
    gib = float(1 << 30)
    fetch_scale = gib / (cf * 1024.0)   # bytes per FETCH_SIZE KiB unit
    write_scale = gib / (cw * 1024.0)
    out = {
        "workload": what,
        "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE, then a separate pass with --pmc WRITE_SIZE "
                  "(tools/gpu_prof.sh); per-dispatch means; units calibrated on a 1 GiB copy (tools/pmc_calib.py)",
        "calibration": {"FETCH_SIZE_per_GiB_read": cf, "WRITE_SIZE_per_GiB_written": cw,
                        "fetch_bytes_per_unit": fetch_scale * 1024.0, "write_bytes_per_unit": write_scale * 1024.0},
    }
    for k in ("pk_step_kernel", "pk_render_kernel"):
        f = fetch.get(k, {}).get("FETCH_SIZE")
        w = write.get(k, {}).get("WRITE_SIZE")
        if f is None or w is None:
            continue
        out[k] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
                  "read_bytes": f * 1024.0 * fetch_scale, "write_bytes": w * 1024.0 * write_scale}
    k1 = out.get("pk_step_kernel")
    out["hbm_bytes_per_launch_k1"] = int(k1["read_bytes"] + k1["write_bytes"]) if k1 else None
    k2 = out.get("pk_render_kernel")
    out["hbm_bytes_per_launch_k2"] = int(k2["read_bytes"] + k2["write_bytes"]) if k2 else None
    out["note"] = ("K1 loads/stores 1 byte per lane (lane-interleaved RAM images); the FETCH calibration is "
                   "for 16-B/lane streams, so the K1 read figure is an upper estimate")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
