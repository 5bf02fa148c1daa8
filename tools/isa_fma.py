"""FP64 contraction A/B at the ISA level: compiles lorb_ba.hip for gfx950 to
assembly twice -- as built (`#pragma clang fp contract(fast)`) and with -DLORB_NO_CONTRACT -- and
prints, per kernel, the FP64 fused multiply-adds (v_fma_f64, v_fmac_f64) against the separate
v_mul_f64 / v_add_f64 instructions.  Static counts (instructions in the code, not executed).

    python tools/isa_fma.py > profiles/r05/fma_isa.txt"""
import os
import re
import subprocess
import sys
import tempfile

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lorb_slam_amd", "csrc", "lorb_ba.hip")
KERNELS = ("k_ba_ls", "k_ba_red", "k_ba_bs2", "k_ba_chol_2s", "k_ba_lin", "k_ba_schur", "k_ba_backsub", "k_ba_pose_only",
           "k_ba_lm_end")


def asm(flags):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "ba.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-ffp-contract=off", *flags, SRC, "-o", out], check=True, cwd=os.path.dirname(SRC),
                       stderr=subprocess.DEVNULL)
        return open(out).read()


def counts(text):
    res = {}
    for m in re.finditer(r"^(_Z\S*):[^\n]*\n(.*?)^\.Lfunc_end", text, re.S | re.M):
        name = m.group(1)
        base = next((k for k in KERNELS if k in name), None)
        if base is None:
            continue
        tpl = re.search(r"ILb([01])E|ILi(\d)E", name)
        key = base + ("<%s>" % (tpl.group(1) or tpl.group(2)) if tpl else "")
        body = m.group(2)
        c = res.setdefault(key, [0, 0, 0])
        c[0] += len(re.findall(r"^\s*v_fmac?_f64", body, re.M))
        c[1] += len(re.findall(r"^\s*v_mul_f64", body, re.M))
        c[2] += len(re.findall(r"^\s*v_add_f64", body, re.M))
    return res


a = counts(asm([]))
b = counts(asm(["-DLORB_NO_CONTRACT"]))
print("kernel                      contract(fast): fma  mul  add | contract off: fma  mul  add")
for k in sorted(set(a) | set(b)):
    x, y = a.get(k, [0, 0, 0]), b.get(k, [0, 0, 0])
    print("%-26s %20d %4d %4d | %17d %4d %4d" % (k, x[0], x[1], x[2], y[0], y[1], y[2]))
sys.stdout.flush()
