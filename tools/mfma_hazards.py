"""MFMA result hazard scanner for the gfx950 code objects in libhvit.so.

An MFMA writes its destination registers several cycles after it issues; an
instruction that touches those registers earlier reads (or clobbers) stale
values.  The hardware does not interlock this: the compiler must pad the gap
with independent instructions or s_nop.  Round 4 found one spot where it did
not (hipcc, ROCm 7.2: the first VALU read of an attention score tile sat 1-3
wait states after its MFMA on a taken branch edge), which
made mhsa_fwd_v2 return wrong, run-to-run different outputs.

This scanner disassembles every gfx950 code object in the library, builds each
function's control-flow graph, and for every MFMA walks EVERY path forward to
the first instruction that touches its destination registers, counting wait
states the way the hazard rules do (one per instruction, N+1 for s_nop N).
An access closer than the MFMA's requirement is a violation, except the next
MFMA of an accumulation chain (same registers as its C operand and result).
It also checks the reverse hazard the compiler pads with s_nop 1: a VALU write
of a register that an MFMA reads within 2 wait states.

Requirements per opcode (wait states between the MFMA and a VALU / VMEM / LDS
read or write of its result, or an MFMA reading it as an A/B operand) are the
ones hipcc itself inserts for gfx950 -- measured by compiling one MFMA
followed by a dependent read per opcode (tools/mfma_hazards.py --probe prints
them again):

    v_mfma_f32_16x16x32_{bf16,f16,fp8/bf8 pairs}        8   (4 passes, XDL)
    v_mfma_f32_32x32x16_{bf16,f16}                      12   (8 passes, XDL)
    v_mfma_scale_f32_16x16x128_f8f6f4                    12 with fp8/bf8 operands, 8 with fp6/fp4
    v_mfma_scale_f32_32x32x64_f8f6f4                     20 with fp8/bf8 operands
    v_mfma_f32_16x16x4_f32                              10   (non-XDL f32)
    v_mfma_f32_32x32x2_f32                              18

    python tools/mfma_hazards.py [path/to/libhvit.so | code-object.elf ...]
"""

from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile
from collections import defaultdict

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# --------------------------------------------------------------- extraction --


def code_objects(path: str) -> list:
    """gfx950 ELF code objects: the library's .hip_fatbin bundles (one per
    translation unit), or the file itself when it already is an ELF."""
    data = open(path, "rb").read()
    if data[:4] == b"\x7fELF" and b".hip_fatbin" not in data:
        return [data]
    if data[:4] == b"\x7fELF":
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "fatbin")
            subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objcopy", f"--dump-section=.hip_fatbin={out}", path,
                            os.path.join(td, "discard")], check=True, capture_output=True)
            data = open(out, "rb").read()
    objs = []
    i = data.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                objs.append(data[i + off:i + off + size])
        i = data.find(MAGIC, i + 1)
    return objs


LINE = re.compile(r"^\s+(?P<ins>[a-z_0-9]+)(?P<ops>[^/]*?)\s*//\s*(?P<addr>[0-9A-Fa-f]+):")
FUNC = re.compile(r"^[0-9a-f]+ <(?P<name>[^>]+)>:")


def disassemble(elf: bytes) -> dict:
    """{function name: [(addr, mnemonic, operand string), ...]}"""
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(elf)
        f.flush()
        out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f.name], check=True, capture_output=True,
                             text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = FUNC.match(line)
        if m:
            cur = funcs.setdefault(m.group("name"), [])
            continue
        m = LINE.match(line)
        if m and cur is not None:
            cur.append((int(m.group("addr"), 16), m.group("ins"), m.group("ops").strip()))
    return funcs


# ------------------------------------------------------------------- model --
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?![\w]))")


def regs(ops: str) -> list:
    """[(file, first, last)] for every VGPR / AGPR operand, in operand order."""
    out = []
    for m in REG.finditer(ops):
        if m.group(2) is not None:
            out.append((m.group(1), int(m.group(2)), int(m.group(3))))
        else:
            r = int(m.group(4))
            out.append((m.group(1), r, r))
    return out


def operands(ops: str) -> list:
    """per comma-separated operand: its register range (file, first, last) or None"""
    out = []
    for tok in ops.split(","):
        m = REG.search(tok.strip().split(" ")[0]) if tok.strip() else None
        if m is None:
            out.append(None)
        elif m.group(2) is not None:
            out.append((m.group(1), int(m.group(2)), int(m.group(3))))
        else:
            out.append((m.group(1), int(m.group(4)), int(m.group(4))))
    return out


def mfma_wait(ins: str, ops: str) -> int:
    """Wait states hipcc puts between this MFMA and a dependent access (gfx950)."""
    if ins.startswith("v_mfma_scale_f32_"):
        fmt = [int(x) for x in re.findall(r"(?:cbsz|blgp):(\d+)", ops)] or [0]
        fp8 = max(fmt) <= 1 or min(fmt) <= 1
        if "32x32x64" in ins:
            return 20 if fp8 else 12
        return 12 if fp8 else 8
    if "32x32x2" in ins and "f32" in ins:
        return 18
    if "16x16x4" in ins and "f32" in ins:
        return 10
    if "32x32" in ins:
        return 12
    return 8


def is_mfma(ins: str) -> bool:
    return ins.startswith("v_mfma")


def waits(ins: str, ops: str) -> int:
    if ins == "s_nop":
        return int(ops.split()[0], 0) + 1
    return 1


def overlap(a, b) -> bool:
    return a[0] == b[0] and a[1] <= b[2] and b[1] <= a[2]


def branch_target(addr: int, ops: str):
    simm = int(ops.split()[0], 0) & 0xFFFF
    if simm >= 0x8000:
        simm -= 0x10000
    return addr + 4 + 4 * simm


def cfg(insts: list):
    """successor lists by instruction index"""
    idx = {a: i for i, (a, _, _) in enumerate(insts)}
    succ = []
    for i, (a, ins, ops) in enumerate(insts):
        s = []
        if ins == "s_endpgm" or ins.startswith("s_setpc") or ins.startswith("s_trap"):
            pass
        elif ins == "s_branch":
            t = idx.get(branch_target(a, ops))
            if t is not None:
                s.append(t)
        elif ins.startswith("s_cbranch"):
            t = idx.get(branch_target(a, ops))
            if t is not None:
                s.append(t)
            if i + 1 < len(insts):
                s.append(i + 1)
        elif i + 1 < len(insts):
            s.append(i + 1)
        succ.append(s)
    return succ


def check_function(name: str, insts: list, limit: int = 24) -> list:
    """Violations in one function: (kind, mfma addr, access addr, distance, need, text)."""
    succ = cfg(insts)
    pred = defaultdict(list)  # (filled below)
    for i, ss in enumerate(succ):
        for j in ss:
            pred[j].append(i)
    out = []
    for i, (a, ins, ops) in enumerate(insts):
        if not is_mfma(ins):
            continue
        od = operands(ops)
        if not od or od[0] is None:
            continue
        dst = od[0]
        srcs = [x for x in od[1:4] if x is not None]
        need = mfma_wait(ins, ops)
        # forward: every path from the MFMA to the first access of its result
        seen = {}
        stack = [(j, 0) for j in succ[i]]
        while stack:
            j, d = stack.pop()
            if d >= need or seen.get(j, 1 << 30) <= d:
                continue
            seen[j] = d
            b_, ins2, ops2 = insts[j]
            if any(overlap(dst, x) for x in regs(ops2)):
                if is_mfma(ins2):
                    o2 = operands(ops2)
                    ab = [x for x in o2[1:3] if x is not None]
                    c2 = o2[3] if len(o2) > 3 else None
                    if any(overlap(dst, x) for x in ab):
                        out.append(("mfma->mfma-ab", a, b_, d, need, f"{ins} {ops}  ->  {ins2} {ops2}"))
                        continue
                    if c2 is not None and overlap(dst, c2) and c2 != dst:
                        out.append(("mfma->mfma-c", a, b_, d, need, f"{ins} {ops}  ->  {ins2} {ops2}"))
                        continue
                    # the result read whole as the next MFMA's C operand (forwarded: hipcc pads
                    # nothing), or only overwritten (the matrix pipe writes in issue order): a
                    # later MFMA writing these registers owns them from here; one that only
                    # reads them as C leaves them to later readers of this MFMA
                    if o2[0] is not None and overlap(dst, o2[0]):
                        continue
                else:
                    out.append(("mfma->access", a, b_, d, need, f"{ins} {ops}  ->  {ins2} {ops2}"))
                    continue
            for k in succ[j]:
                stack.append((k, d + waits(ins2, ops2)))
        # backward: a VALU write of an operand within 2 wait states before the MFMA
        stack = [(j, 0) for j in pred[i]]
        seen = {}
        while stack:
            j, d = stack.pop()
            if d >= 2 or seen.get(j, 1 << 30) <= d:
                continue
            seen[j] = d
            b_, ins2, ops2 = insts[j]
            if ins2.startswith("v_") and not is_mfma(ins2):
                o2 = operands(ops2)
                w = o2[0] if o2 else None
                if w is not None and any(overlap(w, x) for x in srcs):
                    out.append(("valu->mfma", b_, a, d, 2, f"{ins2} {ops2}  ->  {ins} {ops}"))
                    continue
            for k in pred[j]:
                stack.append((k, d + waits(ins2, ops2)))
    return out


def scan(paths) -> tuple:
    """(violations, number of MFMAs checked, number of functions)"""
    viol, nm, nf = [], 0, 0
    for path in paths:
        for co in code_objects(path):
            for name, insts in disassemble(co).items():
                nf += 1
                nm += sum(1 for _, ins, _ in insts if is_mfma(ins))
                for v in check_function(name, insts):
                    viol.append((name,) + v)
    return viol, nm, nf


def probe() -> None:
    """Print the wait states hipcc inserts after each MFMA opcode the library
    uses (the requirement table above)."""
    src = r'''
#include <hip/hip_runtime.h>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16 __attribute__((ext_vector_type(16)));
typedef short s8 __attribute__((ext_vector_type(8)));
typedef int i8 __attribute__((ext_vector_type(8)));
__global__ void a(f4* o, const s8* x) { f4 c = {}; c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[threadIdx.x], x[threadIdx.x+64], c, 0,0,0); o[threadIdx.x] = c * 2.f; }
__global__ void b(f16* o, const s8* x) { f16 c = {}; c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[threadIdx.x], x[threadIdx.x+64], c, 0,0,0); o[threadIdx.x] = c * 2.f; }
__global__ void c(f4* o, const float* x) { f4 c = {}; c = __builtin_amdgcn_mfma_f32_16x16x4f32(x[threadIdx.x], x[threadIdx.x+64], c, 0,0,0); o[threadIdx.x] = c * 2.f; }
__global__ void d(f4* o, const long* x) { f4 c = {}; c = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x[threadIdx.x], x[threadIdx.x+64], c, 0,0,0); o[threadIdx.x] = c * 2.f; }
__global__ void e(f4* o, const i8* x) { f4 c = {}; c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x[threadIdx.x], x[threadIdx.x+64], c, 0, 0, 0, 127, 0, 127); o[threadIdx.x] = c * 2.f; }
__global__ void f(f16* o, const i8* x) { f16 c = {}; c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(x[threadIdx.x], x[threadIdx.x+64], c, 0, 0, 0, 127, 0, 127); o[threadIdx.x] = c * 2.f; }
'''
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "p.hip")
        open(p, "w").write(src)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-c", p, "-o", os.path.join(td, "p.o"),
                        "--save-temps"], cwd=td, check=True, capture_output=True)
        s = open(os.path.join(td, "p-hip-amdgcn-amd-amdhsa-gfx950.s")).read().splitlines()
        for k, line in enumerate(s):
            if "v_mfma" in line:
                n = 0
                for nxt in s[k + 1:]:
                    m = re.match(r"\s+s_nop (\d+)", nxt)
                    if not m:
                        break
                    n += int(m.group(1)) + 1
                ins = line.split()[0]
                print(f"{ins:40s} hipcc pads {n:2d}   table {mfma_wait(ins, line)}")


def main(argv) -> int:
    if argv and argv[0] == "--probe":
        probe()
        return 0
    paths = argv or [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                  "speech-enhancement-via-hybrid-vision-transformer-project_amd", "libhvit.so")]
    viol, nm, nf = scan(paths)
    print(f"scanned {nf} functions, {nm} MFMA instructions: {len(viol)} violations")
    for v in viol[:60]:
        name, kind, a, b, d, need, text = v
        print(f"  {kind:14s} {name[:60]:60s} @{a:x} -> @{b:x}: {d} < {need} wait states   {text}")
    return 1 if viol else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
