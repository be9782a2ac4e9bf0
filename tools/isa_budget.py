#!/usr/bin/env python3
"""Per-component instruction budget of a kernel's sub-step loop, read off
`hipcc -S -gline-tables-only` (DESIGN.md §6 "Instruction budget").

Every instruction in a loop is attributed to the source function whose line
range holds the instruction's `.loc` (the innermost inlined location), and
the functions are grouped into components (Philox-10, Box-Muller, pair force,
BD update, LDS force sums, bookkeeping).  Static counts per loop; the caller
scales them by how often each instance runs per sub-step.

usage: isa_budget.py ASM KERNEL_SUBSTRING [--loops]
  ASM: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -gline-tables-only
       --cuda-device-only -S -o ASM swarmrl_amd/csrc/swarm_engine.hip
"""
import collections
import os
import re
import sys

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "swarmrl_amd", "csrc")

# source function -> component
COMPONENT = {
    "philox4x32_10": "philox",
    "bm_radius": "box_muller", "logf_fixed": "box_muller", "sqrt_pos": "box_muller",
    "group_block": "normals", "normals3": "normals", "normal_from_word": "normals",
    "next": "noise_select",
    "sincos_turn": "sincos",
    "pair_force": "pair_force", "pair_fix_sel": "pair_force", "f2fix24": "pair_force",
    "bd_translate": "bd_update", "bd_step": "bd_update", "advance": "bd_update",
    "i64x2_to_f32": "bd_update", "i64_to_f32": "bd_update", "i64_to_f32_wide": "bd_update",
    "fits_i32": "bd_update", "wave_all2": "bd_update", "wave_all": "bd_update",
    "rcp_rn": "bd_update", "f2i32": "bd_update", "sqrt_rn": "bd_update",
    "wave_lds_sync": "lds_sums",
}


def function_ranges(path):
    """(start, end, name) of each function definition in a source file."""
    defs = []
    pat = re.compile(r"^\s*(?:template\s*<.*>\s*)?(?:__host__\s+)?(?:__device__|__global__)[^(;]*?\b(\w+)\s*\(")
    with open(path) as f:
        lines = f.read().split("\n")
    for k, ln in enumerate(lines, 1):
        m = pat.match(ln)
        if m:
            defs.append((k, m.group(1)))
        m2 = re.match(r"^struct\s+(\w+)", ln)
        if m2:
            defs.append((k, m2.group(1)))
    out = []
    for j, (k, name) in enumerate(defs):
        end = defs[j + 1][0] - 1 if j + 1 < len(defs) else len(lines)
        out.append((k, end, name))
    return out


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    asm, kname = sys.argv[1], sys.argv[2]
    files, ranges = {}, {}
    body = []
    inside = False
    with open(asm) as f:
        for ln in f:
            m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', ln)
            if m:
                files[int(m.group(1))] = m.group(3)
                continue
            if not inside and re.match(r"^_Z\S*%s\S*:" % re.escape(kname), ln):
                inside = True
                continue
            if inside:
                if re.match(r"^\s*\.end_amdhsa_kernel|^\.Lfunc_end", ln):
                    break
                body.append(ln.rstrip("\n"))
    if not body:
        sys.exit("kernel %s not found" % kname)
    for fid, name in files.items():
        p = os.path.join(SRC, name)
        if os.path.exists(p):
            ranges[name] = function_ranges(p)

    def fn_of(fname, line):
        for s, e, n in ranges.get(fname, []):
            if s <= line <= e:
                return n
        return fname

    # basic blocks and loop membership
    loops = collections.OrderedDict()
    cur_loop, cur_loc = None, ("?", 0)
    for ln in body:
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):.*?(?:Header=(BB\S+)|Loop Header)", ln)
        if re.match(r"^(\.LBB\S+|; %bb\.\d+):", ln):
            if "Loop Header" in ln:
                cur_loop = re.match(r"^\.L(BB\S+):", ln).group(1)
            elif m and m.group(2):
                cur_loop = m.group(2)
            else:
                cur_loop = None
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
        if m:
            cur_loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        m = re.match(r"\s+([a-z_][a-z0-9_]*)\b", ln)
        if not m or ln.strip().startswith((".", ";")):
            continue
        if cur_loop is None:
            continue
        op = m.group(1)
        fn = fn_of(*cur_loc)
        comp = COMPONENT.get(fn, "bookkeeping")
        if op.startswith("ds_add") or op.startswith("ds_read") or op.startswith("ds_write") \
                or op.startswith("ds_load") or op.startswith("ds_store"):
            comp = "lds_sums"
        L = loops.setdefault(cur_loop, collections.Counter())
        L[(comp, classify(op))] += 1
        L[("_fn", fn)] += 1
        if op.startswith("v_mad_u64_u32"):
            L[("_mad64", "")] += 1
    for lp, c in loops.items():
        tot = sum(v for (a, b), v in c.items() if not a.startswith("_"))
        print("loop %s: %d instructions" % (lp, tot))
        comps = sorted({a for (a, b) in c if not a.startswith("_")})
        for comp in comps:
            parts = {b: v for (a, b), v in c.items() if a == comp}
            print("  %-13s %4d  %s" % (comp, sum(parts.values()),
                                        " ".join("%s=%d" % kv for kv in sorted(parts.items()))))
        if "--fns" in sys.argv:
            for (a, b), v in sorted(c.items(), key=lambda x: -x[1]):
                if a == "_fn":
                    print("     fn %-24s %d" % (b, v))


if __name__ == "__main__":
    main()
