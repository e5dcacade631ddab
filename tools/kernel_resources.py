#!/usr/bin/env python3
"""Per-kernel resource audit of the built libmsdsp.so (CPU only, no GPU).

Extracts every gfx950 code object from the library's `.hip_fatbin` section (one clang offload
bundle per translation unit), then reads each kernel's metadata note (`llvm-readelf --notes`) and
disassembly (`llvm-objdump -d`).  Per kernel it reports:

* private_segment_fixed_size (scratch bytes per lane) and uses_dynamic_stack;
* sgpr/vgpr spill counts;
* calls (`s_swappc_b64`): an out-of-line device function, whose arguments travel as generic
  (flat) pointers and whose callee-saved registers go to scratch;
* flat memory instructions (`flat_load*`, `flat_store*`, `flat_atomic*`): generic-pointer accesses,
  which reach LDS through the shared aperture and fault outside it;
* scratch instructions.

Round 5's one GPU fault was a build whose live Welch kernel called an out-of-line
numpy pairwise sum through a generic LDS pointer, with 84 B of scratch.  `tests/test_build_check.py`
holds the product kernels to: no calls, no flat memory instructions, no scratch (except the ones
listed there with their reason).

Usage: python tools/kernel_resources.py [path/to/libmsdsp.so] [--json]
"""
from __future__ import annotations

import json
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(data: bytes) -> dict:
    e_shoff = struct.unpack_from("<Q", data, 0x28)[0]
    e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", data, e_shoff + i * e_shentsize) for i in range(e_shnum)]
    stroff = hdrs[e_shstrndx][4]
    out = {}
    for h in hdrs:
        name = data[stroff + h[0]:data.index(b"\0", stroff + h[0])].decode()
        out[name] = (h[4], h[5])  # file offset, size
    return out


def code_objects(so_path: str) -> list[bytes]:
    """The gfx950 code objects inside the library's offload bundles, one per translation unit."""
    data = open(so_path, "rb").read()
    off, size = _sections(data)[".hip_fatbin"]
    fb = data[off:off + size]
    objs = []
    i = 0
    while True:
        j = fb.find(BUNDLE_MAGIC, i)
        if j < 0:
            break
        n = struct.unpack_from("<Q", fb, j + 24)[0]
        p = j + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fb, p)
            triple = fb[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "amdgcn" in triple and esize:
                objs.append(fb[j + eoff:j + eoff + esize])
        i = j + len(BUNDLE_MAGIC)
    return objs


_META_KEYS = ("private_segment_fixed_size", "uses_dynamic_stack", "sgpr_spill_count", "vgpr_spill_count",
              "vgpr_count", "sgpr_count", "group_segment_fixed_size")


def _kernel_metadata(co_path: str) -> dict:
    txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co_path], capture_output=True, text=True,
                         check=True).stdout
    # amdhsa.kernels: one map per kernel, opened by "  - .<first key>", its keys at indent 4
    maps: list = []
    for line in txt.splitlines():
        m = re.match(r"^(  - |    )\.(\w+):\s*(.*)$", line)
        if not m:
            continue
        if m.group(1) == "  - ":
            maps.append({})
        if not maps:
            continue
        key, val = m.group(2), m.group(3).strip()
        if key == "name":
            maps[-1]["name"] = val
        elif key in _META_KEYS:
            maps[-1][key] = val == "true" if val in ("true", "false") else int(val)
    return {k.pop("name"): k for k in maps if "name" in k}


def _function_instructions(co_path: str) -> dict:
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co_path], capture_output=True,
                         text=True, check=True).stdout
    funcs: dict = {}
    cur = None
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
        if m:
            cur = funcs.setdefault(m.group(1), {"calls": 0, "flat": 0, "scratch": 0})
            continue
        if cur is None:
            continue
        s = line.strip()
        op = s.split(None, 1)[0] if s else ""
        if op == "s_swappc_b64":
            cur["calls"] += 1
        elif op.startswith("flat_"):
            cur["flat"] += 1
        elif op.startswith("scratch_"):
            cur["scratch"] += 1
    return funcs


def audit(so_path: str) -> dict:
    """{kernel symbol: resource dict} over every code object of the library."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(so_path)):
            path = os.path.join(td, f"co{k}.o")
            open(path, "wb").write(co)
            meta = _kernel_metadata(path)
            ins = _function_instructions(path)
            for name, m in meta.items():
                r = dict(m)
                r.update(ins.get(name, {"calls": 0, "flat": 0, "scratch": 0}))
                r["code_object"] = k
                out[name] = r
    return out


def _demangle(names):
    try:
        res = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return res.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return list(names)


def main(argv):
    so = next((a for a in argv if not a.startswith("--")),
              os.path.join(os.path.dirname(__file__), "..", "meteor-scatter_amd", "meteorgpu", "libmsdsp.so"))
    res = audit(so)
    if "--json" in argv:
        print(json.dumps(res, indent=1, sort_keys=True))
        return 0
    names = sorted(res)
    for name, dn in zip(names, _demangle(names)):
        r = res[name]
        print(f"{r.get('private_segment_fixed_size', -1):5d} B scratch  dyn={int(r.get('uses_dynamic_stack', 0))} "
              f"spill s/v={r.get('sgpr_spill_count', 0)}/{r.get('vgpr_spill_count', 0)} calls={r['calls']} "
              f"flat={r['flat']} scratch_ops={r['scratch']} vgpr={r.get('vgpr_count', -1)}  {dn[:110]}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
