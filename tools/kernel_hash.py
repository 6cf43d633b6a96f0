"""Hashes of the gfx950 machine code of selected kernels in a built liblidarsm.so.

The committed PMC measurements (profiles/nn_traffic.json, profiles/normals_valu.json) hold for
the machine code they were counted on. A source hash over all of csrc/ is conservative (a change
to the voxel pass or to host code invalidates them); the kernels' own code is what the counters
measured. This script extracts the .so's offload bundles, disassembles them, and hashes each
kernel's instruction text with its addresses made relative (branch targets print as offsets from
the symbol, instruction addresses are dropped), so the hash does not move when other functions
change size.

    python tools/kernel_hash.py LIB.so [name-prefix ...]      (default: the PMC'd kernels)
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
DEFAULT = ("nn_kernel", "nn_fallback_g", "accumulate_kernel", "normals_sparse_kernel",
           "normals_dense_kernel", "normals_refine_kernel")


def demangled_base(sym: str) -> str:
    """'_ZN12_GLOBAL__N_19nn_kernelILb1ELb0EEEv...' -> 'nn_kernel<1,0>'-like readable key."""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)(\w+)", sym)
    if not m:
        return sym
    n = int(m.group(1))
    rest = m.group(1) + m.group(2)
    name = rest[len(m.group(1)):len(m.group(1)) + n]
    tail = rest[len(m.group(1)) + n:]
    targs = re.match(r"I(.*?)EE", tail)
    return name + (f"<{targs.group(1)}>" if targs else "")


def kernel_hashes(lib: str, prefixes=DEFAULT) -> dict:
    tmp = tempfile.mkdtemp(prefix="lsm_khash_")
    try:
        so = os.path.join(tmp, "lib.so")
        shutil.copy(lib, so)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", so], check=True,
                       capture_output=True, cwd=tmp)
        out = {}
        for f in sorted(os.listdir(tmp)):
            if not f.endswith("gfx950"):
                continue
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn",
                                  "--no-leading-addr", os.path.join(tmp, f)],
                                 check=True, capture_output=True, text=True).stdout
            cur, body = None, []

            def flush():
                if cur is not None:
                    base = demangled_base(cur)
                    if any(base.startswith(p) for p in prefixes):
                        text = "\n".join(body)
                        out[base] = hashlib.sha256(text.encode()).hexdigest()[:16]

            for line in dis.splitlines():
                m = re.match(r"^\s*([0-9a-f]+)?\s*<([^>]+)>:\s*$", line)
                if m:
                    flush()
                    cur, body = m.group(2), []
                    continue
                if cur is None:
                    continue
                s = line.strip()
                if not s:
                    continue
                s = re.sub(r"//.*$", "", s).strip()                       # encodings / comments
                s = re.sub(r"<([^>+]+)\+0x([0-9a-f]+)>", r"<+0x\2>", s)    # symbol-relative targets
                s = re.sub(r"\b0x[0-9a-f]{6,}\b", "ADDR", s)                 # absolute addresses
                body.append(s)
            flush()
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    lib = sys.argv[1]
    prefixes = tuple(sys.argv[2:]) or DEFAULT
    print(json.dumps(kernel_hashes(lib, prefixes), indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
