"""Static issue-cost model of a sampler kernel's step loop (no GPU): extracts the kernel's gfx950 ISA from a
libdmip.so and prices every MFMA gap as max(MFMA cycles, 8 + the issue costs of the instructions placed in
it), with MI355X_MICROARCH.md's per-instruction constants (transcendental 8, other VALU / s_nop / LDS / VMEM
issue 4, SALU 1). Prints the modelled cycles between consecutive s_barriers (one per ring chunk), then the whole
step loop (the innermost backward branch enclosing every MFMA of the kernel) with its scratch accesses.
    python scripts/isa_issue_model.py <libdmip.so> <kernel-symbol-substring> [mfma_cycles=16]"""
import re
import subprocess
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
import check_isa  # noqa: E402


def kernel_lines(so, sym):
    for i, o in enumerate(check_isa.code_objects(so)):
        p = f"/tmp/_isa_model_{i}.o"
        open(p, "wb").write(o)
        s = subprocess.run([check_isa.LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn", p],
                           capture_output=True, text=True).stdout
        L = s.splitlines()
        for k, line in enumerate(L):
            if sym in line and line.endswith(">:"):
                out = []
                for l in L[k + 1:]:
                    if l.endswith(">:"):
                        break
                    out.append(l)
                return out
    raise SystemExit(f"{sym} not found")


def cost(op):
    if op.startswith("v_mfma"):
        return None
    if re.match(r"v_(exp|rcp|log|sqrt|rsq|sin|cos)_f32", op):
        return 8
    if op.startswith(("v_", "ds_", "buffer_", "global_", "scratch_")) or op == "s_nop":
        return 4
    return 1


def model(lines, mc):
    gap, tot, pre, n = None, 0, 0, 0
    for l in lines:
        m = re.match(r"\s+([a-z_0-9]+)", l)
        if not m:
            continue
        c = cost(m.group(1))
        if c is None:
            if gap is not None:
                tot += max(mc, gap)
            gap, n = 8, n + 1
        elif gap is None:
            pre += c
        else:
            gap += c
    if gap is not None:
        tot += max(mc, gap)
    return n, tot + pre


def step_loop(L, mc):
    """(MFMAs, modelled cycles, scratch instructions) of the innermost loop that holds every MFMA."""
    addr = []
    for l in L:
        mm = re.search(r"//\s*([0-9A-F]{12}):", l)
        addr.append(int(mm.group(1), 16) if mm else None)
    mf = [i for i, l in enumerate(L) if "v_mfma" in l]
    best = None
    for i, l in enumerate(L):
        mm = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\d+)", l)
        if not mm or addr[i] is None:
            continue
        off = int(mm.group(2))
        off = off - 65536 if off >= 32768 else off
        tgt = addr[i] + 4 + off * 4
        if tgt < addr[i] and tgt in addr:
            j = addr.index(tgt)
            if all(j <= x <= i for x in mf) and (best is None or i - j < best[1] - best[0]):
                best = (j, i)
    if best is None:
        return None
    j, i = best
    n, c = model(L[j:i], mc)
    return n, c, sum(1 for l in L[j:i] if "scratch_" in l)


def main():
    so, sym = sys.argv[1], sys.argv[2]
    mc = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    L = kernel_lines(so, sym)
    bars = [i for i, l in enumerate(L) if "s_barrier" in l]
    tot = 0
    for a, b in zip(bars[1:-1], bars[2:]):
        n, c = model(L[a:b], mc)
        tot += c
        print(f"{a:6d} mfma {n:4d} modelled {c:6d} (floor {n * mc})")
    print("chunks total", tot)
    sl = step_loop(L, mc)
    if sl:
        print(f"step loop: {sl[0]} MFMAs, modelled {sl[1]} cycles, {sl[2]} scratch instructions")


if __name__ == "__main__":
    main()
