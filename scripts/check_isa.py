"""Static checks of libdmip.so's gfx950 code objects (no GPU needed).

Extracts every gfx950 code object from the clang offload bundles embedded in the library and
reports, per kernel: private segment (scratch) bytes per lane, VGPR / AGPR / SGPR counts, LDS bytes,
and whether the kernel body calls an outlined device function (s_swappc). An outlined call puts
register arrays on the scratch stack: that is how a width-512 f32 sampler once faulted on the GPU
(the outlined score evaluation), so the product kernels must have no calls.

    python scripts/check_isa.py [path/to/libdmip.so] [--json]
"""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so_path, arch="gfx950"):
    data = open(so_path, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", data, p)
            ident = data[p + 24:p + 24 + idlen].decode(errors="replace")
            p += 24 + idlen
            if arch in ident and size > 0:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 24)
    return out


def _kernel_meta(elf_path):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", elf_path], capture_output=True, text=True).stdout
    # amdhsa.kernels is a YAML list of maps (keys sorted): a record starts at "  - .<key>:" and its
    # .name may come after other keys of the same record
    recs, cur, in_kernels = [], None, False
    for line in notes.splitlines():
        if re.match(r"^\s*amdhsa\.kernels:", line):
            in_kernels = True
            continue
        if not in_kernels:
            continue
        if re.match(r"^  - \.", line):
            cur = {}
            recs.append(cur)
        m = re.match(r"^\s*(?:- )?\.(name|private_segment_fixed_size|vgpr_count|agpr_count|sgpr_count|"
                     r"group_segment_fixed_size|uses_dynamic_stack):\s+(\S+)", line)
        if m and cur is not None and line.startswith(("  - .", "    .")):
            k, v = m.group(1), m.group(2)
            cur[k] = v if k == "name" else ((v == "true") if v in ("true", "false") else int(v))
    return {r.pop("name"): r for r in recs if "name" in r}


def _calls(elf_path):
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", elf_path], capture_output=True,
                         text=True).stdout
    calls, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            calls.setdefault(cur, 0)
            continue
        if cur and "s_swappc" in line:
            calls[cur] += 1
    return calls


def analyse(so_path):
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(so_path)):
            p = os.path.join(td, f"co{i}.elf")
            open(p, "wb").write(co)
            meta = _kernel_meta(p)
            calls = _calls(p)
            for k, v in meta.items():
                sym = k[:-3] if k.endswith(".kd") else k
                v["calls"] = calls.get(sym, 0)
                res[sym] = v
    return res


def main():
    so = next((a for a in sys.argv[1:] if not a.startswith("--")),
              os.path.join(ROOT, "diffusion-modelling-for-inverse-problems_amd", "libdmip.so"))
    res = analyse(so)
    if "--json" in sys.argv:
        print(json.dumps(res, indent=1, sort_keys=True))
        return
    bad = 0
    for k, v in sorted(res.items()):
        flag = ""
        if v.get("calls", 0) or v.get("private_segment_fixed_size", 0) or v.get("uses_dynamic_stack"):
            flag = "  <-- scratch/calls"
            bad += v.get("calls", 0) > 0 or bool(v.get("uses_dynamic_stack"))
        print(f"{k[:90]:90s} vgpr {v.get('vgpr_count', '?'):>3} agpr {v.get('agpr_count', '?'):>3} "
              f"scratch {v.get('private_segment_fixed_size', '?'):>4} lds {v.get('group_segment_fixed_size', '?'):>6} "
              f"calls {v.get('calls', 0)}{flag}")
    print(f"{len(res)} kernels, {bad} with outlined calls or a dynamic stack")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
