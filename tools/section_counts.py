#!/usr/bin/env python3
"""Static per-phase instruction mix of frame_kernel<NW, false> (diagnostics).

Compiles vp8g_kernels.hip with -DVP8G_MARKS (STAMP(i) -> an asm comment ";MARK_i"), then counts
VALU / SALU / LDS / VMEM / branch instructions between consecutive markers of the chosen
instantiation.  Usage: tools/section_counts.py [NW | quad | quadg] [extra hipcc flags...]
"""
import collections, os, re, subprocess, sys, tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
nw = sys.argv[1] if len(sys.argv) > 1 else "8"
extra = sys.argv[2:]
src = os.path.join(ROOT, "webp-decoder_amd/csrc/vp8g_kernels.hip")
out = os.path.join(tempfile.gettempdir(), "vp8g_marks.s")
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", "-DVP8G_MARKS",
       "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "webp-decoder_amd/csrc"), src, "-o", out] + extra
subprocess.check_call(cmd)
lines = open(out).read().split("\n")
sym = None
for l in lines:
    # NW, or a mangled template-argument fragment such as 16ELb0ELb0ELb1 (the chain kernel)
    # quad: the whole-piece instantiation quad_kernel<16, true>; quadg: the general one
    m = re.match(r"^(_ZN\S*quad_kernelILi16ELb%s\S*):\s*(;.*)?$" % ("1" if nw == "quad" else "0"), l) if nw.startswith("quad") else re.match(r"^(_ZN\S*frame_kernelILi%s\S*):\s*(;.*)?$" % (nw if "E" in nw else nw + "ELb0ELb0ELb0"), l)
    if m:
        sym = m.group(1)
        break
if sym is None:
    sys.exit("instantiation not found")
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith("\t.section") or lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
sec = "pre"
counts = collections.OrderedDict()
def cls(op):
    if op.startswith("v_readlane") or op.startswith("v_writelane"): return "spill"
    if op.startswith("scratch_"): return "scratch"
    if op.startswith("v_") : return "valu"
    if op.startswith("s_cbranch") or op.startswith("s_branch"): return "branch"
    if op.startswith("s_waitcnt") or op.startswith("s_sleep") or op.startswith("s_nop"): return "wait"
    if op.startswith("s_"): return "salu"
    if op.startswith("ds_"): return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"): return "vmem"
    return "other"
for l in body:
    m = re.search(r";MARK_(\d+)", l)
    if m:
        sec = "after_%s" % m.group(1)
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
        continue
    op = t.split()[0]
    counts.setdefault(sec, collections.Counter())[cls(op)] += 1
names = {"pre": "prologue/pair setup", "after_30": "side info+residual+prefetch", "after_0": "wait", "after_1": "borders", "after_2": "predict+bpred",
         "after_3": "save ctx", "after_4": "loop filter", "after_5": "flush", "after_6": "publish/loop"}
print("%-26s %6s %6s %6s %6s %6s %6s %6s %7s" % ("section", "valu", "salu", "branch", "lds", "vmem", "wait", "lanes", "scratch"))
for k, c in counts.items():
    print("%-26s %6d %6d %6d %6d %6d %6d %6d %7d" % (names.get(k, k), c["valu"], c["salu"], c["branch"], c["lds"], c["vmem"], c["wait"], c["spill"],
                                                  c["scratch"]))
