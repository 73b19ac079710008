"""Spilled-SGPR reloads inside the loops of each pathtrace kernel instance (ISA evidence).

With the default --marks, the kernel is compiled with -DRT_ISA_MARKS, which tags the
traversal step, the node step, the leaf batch and the shading step with assembly comments
(RT_ISA_MARK in pathtrace.hip); for each tag the tool reports the innermost loop that
contains it. The markers are volatile asm statements and can move the schedule a little:
read the counts as the product build's to within a few instructions.

The kernels hold more wave-uniform values (kernel arguments, LDS offsets) than the SGPR
file; the compiler parks the rest in lanes of a VGPR (v_writelane) and reloads them with
v_readlane, one VALU instruction each. This tool compiles pathtrace.hip to gfx950
assembly (device only, the build's flags), finds each function's loops (a backward
branch to a label of the same function), and prints per loop: nesting depth, instruction
and VALU counts, and the v_readlane reloads from spill VGPRs (VGPRs written by
v_writelane) inside it.

usage: python tools/isa_loops.py [--kernel SUBSTR] [--asm FILE] [--min-insts N]
"""
import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero", "-fno-slp-vectorize",
         "--cuda-device-only", "-S"]
MARK = re.compile(r"RT_MARK (\w+)")

LABEL = re.compile(r"^(\.?[A-Za-z_$][\w.$]*):")
BRANCH = re.compile(r"^\s+s_(?:cbranch_\w+|branch)\s+(\S+)")
INST = re.compile(r"^\s+([a-z_][a-z0-9_]*)")
WRITELANE = re.compile(r"^\s+v_writelane_b32\s+(v\d+),")
READLANE = re.compile(r"^\s+v_readlane_b32\s+s\[?\d+(?::\d+\])?,\s*(v\d+),")


def compile_asm(out: Path, marks: bool):
    cmd = ["/opt/rocm/bin/hipcc", *FLAGS, *(["-DRT_ISA_MARKS"] if marks else []), "-o", str(out), "-I", str(ROOT / "include"),
           "-I", str(ROOT / "rust_gpu_raytracing_amd/csrc"), str(ROOT / "rust_gpu_raytracing_amd/csrc/pathtrace.hip")]
    subprocess.run(cmd, check=True)


def functions(lines):
    """Yield (name, body lines) for each kernel/function in the assembly."""
    name, body = None, []
    for ln in lines:
        m = LABEL.match(ln)
        if m and not m.group(1).startswith("."):  # a function's own label (block labels are .LBB*)
            if name is not None:
                yield name, body
            name, body = m.group(1), []
            continue
        if name is not None:
            if ln.strip().startswith(".Lfunc_end"):
                yield name, body
                name, body = None, []
            else:
                body.append(ln)
    if name is not None:
        yield name, body


def analyse(body):
    labels = {}
    insts = []  # (line index, mnemonic)
    for i, ln in enumerate(body):
        m = LABEL.match(ln)
        if m:
            labels[m.group(1)] = i
            continue
        mi = INST.match(ln)
        if mi and not ln.strip().startswith(";") and not ln.strip().startswith("."):
            insts.append((i, mi.group(1)))
    spill = set()
    for ln in body:
        w = WRITELANE.match(ln)
        if w:
            spill.add(w.group(1))
    loops = []
    for i, ln in enumerate(body):
        b = BRANCH.match(ln)
        if b and b.group(1) in labels and labels[b.group(1)] < i:
            loops.append((labels[b.group(1)], i))
    loops = sorted(set(loops))
    out = []
    for lo, hi in loops:
        depth = sum(1 for a, b in loops if a <= lo and hi <= b and (a, b) != (lo, hi))
        inner = not any(lo <= a and b <= hi and (a, b) != (lo, hi) for a, b in loops)
        n = valu = rl = 0
        for i, mn in insts:
            if lo <= i <= hi:
                n += 1
                if mn.startswith("v_"):
                    valu += 1
                if mn == "v_readlane_b32":
                    r = READLANE.match(body[i])
                    if r and r.group(1) in spill:
                        rl += 1
        out.append(dict(depth=depth, innermost=inner, insts=n, valu=valu, spill_readlanes=rl, first=lo, last=hi))
    total_rl = sum(1 for ln in body if (lambda r: r and r.group(1) in spill)(READLANE.match(ln)))
    marks = {}
    for i, ln in enumerate(body):
        mk = MARK.search(ln)
        if mk:
            inside = [lp for lp in out if lp["first"] <= i <= lp["last"]]
            if inside:
                best = min(inside, key=lambda lp: lp["last"] - lp["first"])
                marks.setdefault(mk.group(1), best)
    return spill, out, total_rl, marks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="rt_pathtrace_kernel")
    ap.add_argument("--asm", default="", help="analyse this assembly file instead of compiling")
    ap.add_argument("--min-insts", type=int, default=40, help="omit loops smaller than this (--all-loops)")
    ap.add_argument("--all-loops", action="store_true", help="list every loop, not only the marked ones")
    ap.add_argument("--no-marks", action="store_true", help="compile without the region markers")
    args = ap.parse_args()
    if args.asm:
        text = Path(args.asm).read_text()
    else:
        with tempfile.TemporaryDirectory() as d:
            out = Path(d) / "pathtrace.s"
            compile_asm(out, not args.no_marks)
            text = out.read_text()
    for name, body in functions(text.splitlines()):
        if args.kernel not in name:
            continue
        spill, loops, total_rl, marks = analyse(body)
        short = re.sub(r"_Z19rt_pathtrace_kernelILi(\d)ELj(\d+)ELb([01])ELb([01])EEv10KernelArgs",
                       r"pathtrace<mode \1, \2 threads, tris \3, wide \4>", name)
        print(f"{short}: spill VGPRs {sorted(spill)}, spill reloads in the kernel {total_rl}")
        for tag, lp in sorted(marks.items()):
            print("  {tag:10s} innermost loop around it: insts {insts:5d} valu {valu:5d} spill_readlanes {spill_readlanes:3d}".format(
                tag=tag, **lp))
        for lp in loops if args.all_loops else []:
            if lp["insts"] < args.min_insts:
                continue
            print("  loop depth {depth} {kind:9s} insts {insts:5d} valu {valu:5d} spill_readlanes {spill_readlanes:3d}".format(
                kind="innermost" if lp["innermost"] else "", **lp))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
