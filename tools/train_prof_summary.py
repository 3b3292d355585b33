"""Per-pass summary of the fp32 training convolutions from a rocprofv3 kernel trace of
tools/probe_train.py (gpu_session.sh step prof_train): for each pass, the dispatches at the
PPO minibatch size (16,384 samples; the rollout's 4,096-env forwards of the same kernels run
~4x shorter and are split off by duration), their mean duration, and the algorithmic
TFLOP/s against the 157.3 TF fp32 matrix peak.  The weight-gradient passes include their
fixed-order partial reduce.  Also: the Solver update's other kernels by total time.

    python tools/train_prof_summary.py gpurun_out/<tag>/prof_train/train_kernel_trace.csv [--out x.json]
"""
import argparse
import collections
import csv
import json

PEAK = 157.3
N = 16384
FLOP = {1: 2 * N * 400 * 32 * 27, 2: 2 * N * 400 * 64 * 288, 3: 2 * N * 400 * 64 * 576}
PASSES = {  # kernel name fragment -> (pass, layer)
    "conv_a_kernel<4, 32, 1, 0": ("conv1_fwd", 1),
    "conv_a_kernel<32, 64, 1, 0": ("conv2_fwd", 2),
    "conv_a_kernel<64, 64, 1, 0": ("conv3_fwd", 3),
    "conv_a_kernel<64, 64, 1, 1": ("conv3_dgrad", 3),
    "conv_a_kernel<64, 32, 2, 1": ("conv2_dgrad", 2),
    "conv_w_kernel<64, 64": ("conv3_wgrad", 3),
    "conv_w_kernel<32, 64": ("conv2_wgrad", 2),
    "conv_w_kernel<4, 32": ("conv1_wgrad", 1),
    "conv_w_reduce_kernel<64, 64": ("conv3_wgrad_reduce", 3),
    "conv_w_reduce_kernel<32, 64": ("conv2_wgrad_reduce", 2),
    "conv_w_reduce_kernel<4, 32": ("conv1_wgrad_reduce", 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    a = ap.parse_args()
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res, other = {}, {}
    for name, d in durs.items():
        key = next((k for k in PASSES if k in name), None)
        if key is None:
            other[name] = sum(d)
            continue
        p, layer = PASSES[key]
        big = max(d)
        mb = [x for x in d if x > 0.6 * big]  # the minibatch-size dispatches
        res[p] = {"calls": len(mb), "mean_us": sum(mb) / len(mb), "rollout_size_calls": len(d) - len(mb)}
    for p in list(res):
        if p.endswith("_reduce"):
            continue
        layer = next(l for k, (q, l) in PASSES.items() if q == p)
        us = res[p]["mean_us"] + res.get(p + "_reduce", {}).get("mean_us", 0.0)
        res[p]["us_with_reduce"] = us
        res[p]["tflops"] = FLOP[layer] / (us * 1e-6) / 1e12
        res[p]["frac_fp32_matrix_peak"] = res[p]["tflops"] / PEAK
    tot = sum(v.get("us_with_reduce", 0.0) for v in res.values())
    out = {"minibatch": N, "peak_tflops": PEAK, "passes": res, "sum_us_per_minibatch_step": tot,
           "flop_per_minibatch_step": 3 * sum(FLOP.values()) - FLOP[1],
           "other_kernels_top_ms": {k[:120]: v / 1e3 for k, v in sorted(other.items(), key=lambda kv: -kv[1])[:15]}}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
