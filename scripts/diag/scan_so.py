"""Disassemble every gfx950 code object inside a built library (_C.so) and report, per kernel, the MFMA count and
the packed-FP32 instructions that take the HIGH half of src1 through op_sel (v_pk_*_f32 ... op_sel:[x,1...]).

Round 3 (profiles/afno_o3_bisect_r3.txt, scripts/diag/opsel_lds_repro.hip): on MI355X those instructions return wrong
results while another wave on the same SIMD executes MFMAs, so a kernel must not contain both (and a kernel that
contains only the packed form must never share a SIMD with MFMA work).

  python scripts/diag/scan_so.py [tensorrt_dft_plugins_amd/_C.so]     (exit 1 if a kernel contains both)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
SRC1HI = re.compile(r"^\s*v_pk_\w+_f32\b.*op_sel:\[[01],1")


def code_objects(so, tmp):
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", so, os.path.join(tmp, "x")],
                   check=True, capture_output=True)
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for i, s in enumerate(starts):
        chunk = data[s:starts[i + 1] if i + 1 < len(starts) else len(data)]
        b = os.path.join(tmp, f"b{i}")
        open(b, "wb").write(chunk)
        o = os.path.join(tmp, f"co{i}")
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                            f"--output={o}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(o) > 0:
            out.append(o)
    return out


def scan(so):
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(so, tmp):
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                                 capture_output=True, text=True).stdout
            fn = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    fn = m.group(1)
                    res.setdefault(fn, [0, 0])
                    continue
                if fn is None:
                    continue
                if "v_mfma" in line:
                    res[fn][0] += 1
                elif SRC1HI.search(line):
                    res[fn][1] += 1
    return res


if __name__ == "__main__":
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "..", "tensorrt_dft_plugins_amd", "_C.so")
    r = scan(so)
    both = {k: v for k, v in r.items() if v[0] and v[1]}
    print(f"{len(r)} kernels; with MFMA {sum(1 for v in r.values() if v[0])}; with packed src1-high op_sel "
          f"{sum(1 for v in r.values() if v[1])}; with both {len(both)}")
    for k, (m, p) in sorted(r.items()):
        if p:
            print(f"  src1-high packed x{p:4d}  mfma x{m:5d}  {k[:110]}")
    sys.exit(1 if both else 0)
