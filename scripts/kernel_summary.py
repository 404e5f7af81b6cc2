"""Summarise a rocprofv3 --stats run: top kernels by total time with short names."""
import csv
import glob
import re
import sys


def short(n: str) -> str:
    m = re.search(r"fft_fixed_kernel<\(amd_dft::Kind\)(\d), (\w+), (\d+), (\d+), amd_dft::fixed_detail::FL<(.*?)>", n)
    if m:
        return f"fft_fixed K{m.group(1)} cols={m.group(2)} TP={m.group(3)} T={m.group(4)} R=<{m.group(5)}>"
    m = re.search(r"gemm_bf16_kernel<(.*?)>", n)
    if m:
        return "gemm<" + m.group(1).replace("true", "T").replace("false", "F") + ">"
    for k in ("afno_spectral_x3_kernel", "afno_spectral_kernel", "afno_w_r2c_ln_kernel", "afno_w_c2r_ln_kernel", "ln_f32_kernel", "split_bf16_kernel", "ln_bf16_kernel", "fft_pass_kernel", "fno_mix", "fno_pointwise_kernel", "patch_remap", "fno_c2r_pw_kernel", "dftw_r2c_kernel", "gemm_bf16_kernel", "ln_stats_kernel"):
        if k in n:
            return k + (n[n.index(k) + len(k):][:40])
    return n[:110]


def main():
    d = sys.argv[1]
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot/1e6:.2f} ms")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        print(f"{float(r['Percentage']):6.2f}%  {float(r['TotalDurationNs'])/1e6:9.3f} ms  n={r['Calls']:>5}  "
              f"avg={float(r['AverageNs'])/1e3:9.1f} us  {short(r['Name'])}")


if __name__ == "__main__":
    main()
