"""Static instruction mix of k_accumulate's hot loop (the one-entry mixed-add block) and the VALU
issue cycles it demands per wave-iteration on gfx950.

    python tools/isa_mix.py --asm <device .s> --lib <libmsm.so> --out <libmsm.isa.json>   (make)
    python tools/isa_mix.py --out <json>          (compiles its own copy with --save-temps)

The Makefile builds libmsm.so with -save-temps and runs this on the device assembly of that same
compile, recording the shipped library's sha256: the assembly is what the code object inside
that .so was assembled from, so bench.py's ISA floor belongs to the library it loads (it checks
the hash and reports no floor on a mismatch).  The basic block of k_accumulate holding the most
64-bit multiply-adds (one pt_madd per wave-iteration) is priced two ways:
  * cycles_per_iteration: the nominal gfx950 model (a SIMD-32 issues a 32-bit VALU wave64
    instruction in 2 cycles, a 64-bit one -- v_mad_u64_u32, 64-bit shifts/adds/moves -- in 4);
  * ns_per_iteration_chip: every instruction at the chip-wide issue rate MEASURED for it (or its
    encoding class) by tools/ubench/isa_rates.hip (profiles/r2_isa_rates.json, G wave-instructions
    per second over all 256 CUs), so clock and encoding effects are in the price.
bench.py turns these into the ISA floor of the kernel: floor = (entries / 64) x ns_per_iteration_chip,
frac_isa_measured = floor / k_accumulate duration.

The loop's other blocks are priced too (`loop_classes`), by what runs them: the blocks every
wave-iteration passes (loop header, exec-mask joins, the entry select), the sorted-entry vector
load (every fourth iteration), and the bucket-boundary path -- the finished bucket's store, the
accumulator reset and the advance to the next bucket (a wave runs it whenever ANY of its 64 lanes
reaches a bucket end) and the run head's LDS staging (a lane's first bucket end).  bench.py weights
them by their execution frequency for the launch's entries and buckets and adds
them to the floor.
"""
import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "webgpu-msm_amd", "csrc", "msm_host.hip")
MADS = ("v_mad_u64_u32", "v_mad_i64_i32")
VALU64 = {"v_mad_u64_u32", "v_mad_i64_i32", "v_lshrrev_b64", "v_lshlrev_b64", "v_lshl_add_u64", "v_mov_b64",
          "v_add_u64", "v_ashrrev_i64", "v_fma_f64"}


def asm_text(tmp):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared", "--save-temps",
           "-Xarch_host", "-mbmi2", "-Xarch_host", "-madx", "-o", os.path.join(tmp, "lib.so"), SRC]
    subprocess.run(cmd, cwd=tmp, check=True, capture_output=True)
    with open(os.path.join(tmp, "msm_host-hip-amdgcn-amd-amdhsa-gfx950.s")) as f:
        return f.read()


def blocks_of(asm, func):
    """{block: [opcodes]} of `func`, and the blocks of its loops (the assembler's "in Loop" /
    "Loop Header" annotations on the label line or the comment lines right after it)."""
    blocks, depth = basic_blocks(asm, func)
    return blocks, {b for b, d in depth.items() if d >= 1}


def basic_blocks(asm, func):
    """Basic blocks split at every label (.LBB) and fall-through block comment (; %bb.N:), with
    each block's loop depth (0 outside loops)."""
    lines = asm.splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(func + ":"))
    out, depth, cur, head = {}, {}, None, False
    for l in lines[start:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\w+|" + func + r"):", l) or re.match(r"^; (%bb\.\d+):", l)
        if m:
            cur = m.group(1)
            out[cur], depth[cur], head = [], 0, True
        s = l.strip()
        if head and ";" in l:  # the label line's annotation, then comment-only lines after it
            d = re.search(r"Depth=(\d+)", l)
            if d:
                depth[cur] = max(depth[cur], int(d.group(1)))
            elif "Loop" in l:
                depth[cur] = max(depth[cur], 1)
            if not m and not s.startswith(";"):
                head = False
        elif not m:
            head = False
        if cur and s and not s.startswith((";", ".")) and not m:
            out[cur].append(s.split()[0])
            if s.startswith("s_cbranch") or s.startswith("s_branch"):
                TARGETS.setdefault(cur, set()).add(s.split()[-1])
    return out, depth


TARGETS = {}  # block -> labels it branches to (filled by basic_blocks)


def classify_loop(blocks, depth, main, targets=None):
    """Classes of the depth-1 loop blocks other than the main (mixed-add) block, by what they hold:
    'boundary' (bucket-end store, accumulator reset: >= 18 moves, advance), 'head' (LDS staging of a
    run's head), 'vecload' (the every-fourth-iteration entry load), 'gallop' (the inner search
    loops over empty buckets, depth 2), 'iteration' (everything else: every wave-iteration)."""
    targets = targets or {}
    cls = {}
    for b, ops in blocks.items():
        if b == main or depth.get(b, 0) < 1:
            continue
        if depth[b] >= 2:
            cls[b] = "gallop"
        elif any(o.startswith("ds_write") for o in ops):
            cls[b] = "head"
        elif any(o.startswith("global_store") for o in ops):
            cls[b] = "boundary"
        elif sum(1 for o in ops if o.startswith("v_mov_b32")) >= 18:
            cls[b] = "boundary"  # the accumulator reset to the identity
        elif any(o.startswith("global_load_dwordx4") for o in ops):
            cls[b] = "vecload"
        elif any(o == "global_load_dword" for o in ops):
            # one-word loads outside the mixed add: the per-entry load of runs that are not 16-B
            # aligned (it branches straight back into the main block; unused when K % 4 == 0), or
            # the search over empty buckets (rare with random scalars)
            cls[b] = "scalar_entry" if main in targets.get(b, ()) else "gallop"
        else:
            cls[b] = "iteration"
    return cls


# instructions the rate benchmark does not time, priced as the measured instruction of their
# encoding class (VOP2 32-bit ~ v_and_b32, VOP3 32-bit ~ v_add3_u32, 64-bit shifts ~ v_lshrrev_b64)
RATE_CLASS = {"v_sub_u32": "v_add_u32", "v_add_u32": "v_add_u32", "v_lshrrev_b32": "v_and_b32",
              "v_lshlrev_b32": "v_and_b32", "v_or_b32": "v_and_b32", "v_xor_b32": "v_and_b32",
              "v_mov_b32": "v_and_b32", "v_not_b32": "v_and_b32", "v_bitop3_b32": "v_add3_u32",
              "v_bfi_b32": "v_add3_u32", "v_lshl_or_b32": "v_add3_u32", "v_and_or_b32": "v_add3_u32",
              "v_or3_b32": "v_add3_u32", "v_lshlrev_b64": "v_lshrrev_b64", "v_ashrrev_i64": "v_lshrrev_b64",
              "v_add_co_u32": "v_and_b32", "v_addc_co_u32": "v_and_b32", "v_sub_co_u32": "v_and_b32",
              "v_subb_co_u32": "v_and_b32", "v_perm_b32": "v_add3_u32", "v_mul_lo_u32": "v_mul_lo_u32",
              "v_mul_hi_u32": "v_mul_hi_u32"}


def price_measured(cnt, rates_path):
    """Chip-wide ns per wave-iteration (one wave of every SIMD... i.e. per 1 wave-instruction
    stream) from the measured issue rates; returns (ns, unpriced ops)."""
    with open(rates_path) as f:
        rates = json.load(f)["rates"]
    ns, unpriced = 0.0, {}
    for op, c in cnt.items():
        if not op.startswith("v_"):
            continue  # scalar / memory / waitcnt: not VALU issue
        key = op if op in rates else RATE_CLASS.get(op)
        if key is None and op.startswith("v_cmp"):
            key = "v_and_b32"
        if key is None or key not in rates:
            unpriced[op] = c
            key = "v_add3_u32"
        ns += c / rates[key]["G_wave_inst_per_s"]  # G/s -> ns per wave-instruction, chip-wide
    return ns, unpriced


def base(op):
    return re.sub(r"_e(32|64)$", "", op)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "webgpu-msm_amd", "msm_amd", "_lib", "libmsm.isa.json"))
    ap.add_argument("--func", default="k_accumulate")
    ap.add_argument("--rates", default=os.path.join(ROOT, "profiles", "r2_isa_rates.json"))
    ap.add_argument("--asm", help="device assembly of the library build (-save-temps); default: compile a copy")
    ap.add_argument("--lib", help="the library that assembly was linked into (its sha256 is recorded)")
    args = ap.parse_args()
    if args.asm:
        with open(args.asm) as f:
            asm = f.read()
    else:
        with tempfile.TemporaryDirectory() as tmp:
            asm = asm_text(tmp)
    blocks, loops = blocks_of(asm, args.func)
    _, depth = basic_blocks(asm, args.func)
    # the loop block with the most multiplies: one entry's pt_madd per wave-iteration
    name, ins = max(((k, v) for k, v in blocks.items() if k in loops),
                    key=lambda kv: sum(1 for o in kv[1] if o in MADS))
    # The record gather (seven loads per entry) belongs to the same wave-iteration; if the compiler
    # splits it into a loop block of its own, count that block too, so a split cannot shrink the
    # per-entry figure.
    def nloads(v):
        return sum(1 for o in v if o.startswith(("global_load", "buffer_load")))
    merged = [name]
    if nloads(ins) < 7:
        rest = [(k, v) for k, v in blocks.items() if k in loops and k != name]
        if rest:
            g = max(rest, key=lambda kv: nloads(kv[1]))
            if nloads(g[1]) >= 7:
                ins = ins + g[1]
                merged.append(g[0])
    cnt = collections.Counter(base(o) for o in ins)
    v64 = sum(c for o, c in cnt.items() if o in VALU64)
    v32 = sum(c for o, c in cnt.items() if o.startswith("v_") and o not in VALU64)
    cycles = 4 * v64 + 2 * v32
    res = {"kernel": args.func, "block": name, "blocks": merged, "instructions": len(ins), "valu64": v64, "valu32": v32,
           "v_mad_u64_u32": cnt["v_mad_u64_u32"], "v_mad_i64_i32": cnt["v_mad_i64_i32"],
           "vmem_loads": sum(c for o, c in cnt.items() if o.startswith(("global_load", "buffer_load"))),
           "cycles_per_iteration": cycles,
           "cycle_model": "gfx950 SIMD-32: 2 cycles per 32-bit VALU wave64 instruction, 4 per 64-bit one "
                          "(v_mad_u64_u32, 64-bit shifts/adds/moves); profiles/r2_isa_rates.json",
           "mix": dict(cnt.most_common())}
    if args.lib:
        import hashlib
        with open(args.lib, "rb") as f:
            res["lib_sha256"] = hashlib.sha256(f.read()).hexdigest()
        res["lib"] = os.path.basename(args.lib)
    # the loop's other blocks, by class (priced below when the rates file is present)
    cls = classify_loop(blocks, depth, name, TARGETS)
    classes = {}
    for b, k in cls.items():
        if b in merged:
            continue
        c = classes.setdefault(k, {"blocks": [], "instructions": 0, "valu": 0, "mix": collections.Counter()})
        c["blocks"].append(b)
        c["instructions"] += len(blocks[b])
        c["valu"] += sum(1 for o in blocks[b] if o.startswith("v_"))
        c["mix"].update(base(o) for o in blocks[b])
    if os.path.exists(args.rates):
        for k, c in classes.items():
            c["ns_chip"], _ = price_measured(c["mix"], args.rates)
    for c in classes.values():
        c["mix"] = dict(c["mix"].most_common())
    res["loop_classes"] = classes
    if os.path.exists(args.rates):
        ns, unpriced = price_measured(cnt, args.rates)
        res["ns_per_iteration_chip"] = ns
        res["rates_file"] = os.path.relpath(args.rates, ROOT)
        res["measured_model"] = ("sum over the block's VALU instructions of 1 / (chip-wide measured issue rate of the "
                                 "instruction or its encoding class): ns of chip time per wave-iteration when every "
                                 "SIMD issues back to back")
        if unpriced:
            res["unpriced_as_vop3"] = unpriced
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "mix"}))


if __name__ == "__main__":
    main()
