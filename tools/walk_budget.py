"""Instruction budget of the normals' walk loops, from the gfx950 machine code of the built library.

VERDICT r4 item 3 asks for the instructions per walk step of normals_dense_kernel<4>'s scan 1 and
final pass. This disassembles the kernel (llvm-objdump over the .so's offload bundle, as
tools/kernel_hash.py), finds its loops (backward branches) and reports, for the innermost loops
that walk points (they hold buffer loads of points: 4 per trip with G = 4), the instructions per
trip split into

  * always issued: outside every `s_cbranch_execz`-guarded region (the wave runs them whenever
    it runs the trip);
  * guarded: inside such regions (skipped when no lane of the wave takes them), split into the
    regions that hold f64 arithmetic (the exact-distance bands, the cumulant adds) and the rest
    (e.g. the LDS histogram add);

each as VALU / SALU / f64 / memory counts, and per point step (/ G).

    python tools/walk_budget.py [LIB.so] [--kernel normals_dense_kernel] [--json OUT]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(lib: str, kernel: str) -> list:
    """[(addr, opcode, operands, branch target or None)] of the first symbol matching `kernel`."""
    tmp = tempfile.mkdtemp(prefix="lsm_walk_")
    try:
        so = os.path.join(tmp, "lib.so")
        shutil.copy(lib, so)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", so], check=True,
                       capture_output=True, cwd=tmp)
        for f in sorted(os.listdir(tmp)):
            if not f.endswith("gfx950"):
                continue
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn",
                                  os.path.join(tmp, f)], check=True, capture_output=True,
                                 text=True).stdout
            out, cur, base = [], False, None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <([^>]+)>:\s*$", line)
                if m:
                    if cur:
                        return out
                    cur = kernel in m.group(1) and "ILi4E" in m.group(1)
                    continue
                if not cur:
                    continue
                m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):.*?(<[^>]*\+0x([0-9a-f]+)>)?\s*$",
                             line)
                if not m:
                    continue
                a = int(m.group(3), 16)
                base = a if base is None else base
                tgt = base + int(m.group(5), 16) if m.group(5) else None
                out.append((a, m.group(1), m.group(2), tgt))
            if out:
                return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    raise SystemExit(f"kernel {kernel} not found in {lib}")


def kind(op: str) -> str:
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def budget(ins, j, k):
    """Counts of the trip [j, k] split by execz-guarded regions."""
    pos = {a: i for i, (a, *_r) in enumerate(ins)}
    guarded = [None] * (k - j + 1)   # None: always; "f64" / "plain": inside a guarded region
    for i in range(j, k + 1):
        a, op, arg, t = ins[i]
        if op == "s_cbranch_execz" and t is not None and t > a and t in pos and pos[t] <= k:
            e = pos[t]
            f64 = any("f64" in ins[q][1] for q in range(i + 1, e))
            for q in range(i + 1, e):
                if guarded[q - j] is None or f64:
                    guarded[q - j] = "f64" if f64 else (guarded[q - j] or "plain")
    res = {}
    for cls in (None, "plain", "f64"):
        c = {"valu": 0, "salu": 0, "f64": 0, "vmem": 0, "lds": 0}
        for q in range(j, k + 1):
            if guarded[q - j] != cls:
                continue
            kd = kind(ins[q][1])
            if kd in c:
                c[kd] += 1
            if ins[q][1].startswith("v_") and "f64" in ins[q][1]:
                c["f64"] += 1
        res["always" if cls is None else f"guarded_{cls}"] = c
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(ROOT, "lidar_slam_arvc_amd", "_lib",
                                                          "liblidarsm.so"))
    ap.add_argument("--kernel", default="normals_dense_kernel")
    ap.add_argument("--group", type=int, default=4, help="points per walk trip (G)")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    ins = disassemble(args.lib, args.kernel)
    pos = {a: i for i, (a, *_r) in enumerate(ins)}
    loops = []
    for k, (a, op, arg, t) in enumerate(ins):
        if t is not None and t <= a and (op.startswith("s_cbranch") or op == "s_branch"):
            loops.append((pos[t], k))
    walks = []
    for j, k in sorted(set(loops)):
        pts = sum(1 for q in range(j, k + 1)
                  if ins[q][1].startswith("buffer_load_dwordx3") or
                  ins[q][1].startswith("buffer_load_dwordx4"))
        inner = not any(j < j2 and k2 < k and (j2, k2) != (j, k) for j2, k2 in loops)
        if pts >= args.group and inner:
            has_hist = any(ins[q][1] == "ds_add_u32" for q in range(j, k + 1))
            nf64 = sum(1 for q in range(j, k + 1) if "f64" in ins[q][1])
            walks.append({"offset": f"0x{ins[j][0] - ins[0][0]:x}", "instructions": k - j + 1,
                          "point_loads": pts,
                          "role": ("scan 1 (histogram)" if has_hist else
                                   "final pass / refine (f64 cumulants)" if nf64 >= 24 else
                                   "other walk"),
                          "per_trip": budget(ins, j, k)})
    for w in walks:
        w["per_point_step"] = {cls: {kk: round(v / args.group, 2) for kk, v in c.items()}
                               for cls, c in w["per_trip"].items()}
    out = {"kernel": f"{args.kernel}<4>", "group_points_per_trip": args.group, "walks": walks}
    text = json.dumps(out, indent=1)
    print(text)
    if args.json:
        with open(args.json, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    sys.exit(main())
