"""One-screen summary of a bench.py output file (the JSON line among RCCL banner lines).
    python tools/bench_summary.py gpurun_out/TAG/bench_N.json"""
import json
import sys


def main():
    line = [ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1]
    d = json.loads(line)
    r = d["roofline"]
    print(f"value {d['value']} Mpix/s  ms/step {d['ms_per_step']}  kernel {d['kernels']}  frac {r['frac']}"
          f"  traffic {r['traffic']}")
    if d.get("roundtrip"):
        k = d["roundtrip"]["kernels"]["pipeline_r2h_h2r"]
        print(f"roundtrip {k['ms']} ms frac {k['frac_of_peak']}  unfused {d['roundtrip']['unfused']['ms_per_step']} ms")
    if d.get("pyramid"):
        p = d["pyramid"]
        print(f"pyramid {p['ms_per_step']} ms frac {p['frac_of_peak']}  levels "
              f"{[v['ms'] for v in p['kernels'].values()]}  unfused {p['unfused']['ms_per_step']} ms")
    if d.get("unfused"):
        print("unfused", {k: v["ms"] for k, v in d["unfused"]["kernels"].items()}, d["unfused"]["ms_per_step"])
    if d.get("wide_conv"):
        print("wide", d["wide_conv"]["ms"], d["wide_conv"]["TFLOP_s"], d["wide_conv"]["roofline"]["frac"])
    if d.get("lattices"):
        print("lattices", {k: (v["ms"], v["frac_of_peak"]) for k, v in d["lattices"].items()})
    if d.get("cpu_baseline"):
        print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])


if __name__ == "__main__":
    main()
