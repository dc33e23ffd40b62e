"""Per-kernel gfx950 ISA of one HIP source, for "this change leaves the existing kernels' code unchanged"
checks (round 6: the 16-bit format templates of llama_kernels.hip / attn_kernels.hip).

    python scripts/diag/isa_compare.py dump <src.hip> <out.json>      # kernel -> normalised instructions
    python scripts/diag/isa_compare.py diff <before.json> <after.json> [--map OLD=NEW ...]

``--re PATTERN=REPL`` applies a regular-expression substitution instead.

``dump`` compiles the source to device assembly with the library's flags and keeps, per kernel
symbol, its instruction lines with basic-block labels and comments stripped (labels are renumbered
between builds). ``diff`` pairs kernels by demangled name after applying ``--map`` substitutions
(a template parameter added with its old value, e.g. ``--map "<4, false>=<4, false, 0>"``) and prints
identical / differing / unmatched kernels. Exit status 1 when any paired kernel differs."""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def dump(src, out):
    from sparse_matrix_tuning_amd import build
    flags = build.FILE_FLAGS.get(os.path.basename(src), [])
    with tempfile.TemporaryDirectory() as d:
        s = os.path.join(d, "k.s")
        cmd = [build.hipcc(), f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-function",
               "-I", os.path.join(ROOT, "include"), *flags, "--cuda-device-only", "-S", "-o", s, src]
        subprocess.run(cmd, check=True)
        text = open(s).read()
    kernels, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^([_A-Za-z][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith((".L", "$")):
            cur = m.group(1)
            kernels[cur] = []
            continue
        if cur is None:
            continue
        if line.startswith(("\t.end_amdhsa_kernel", ".Lfunc_end", "\t.section", "\t.amdgpu_metadata")):
            cur = None
            continue
        ins = line.split(";")[0].strip()
        if not ins or ins.startswith(".") or re.match(r"^\.?L\w+:", ins):
            continue
        kernels[cur].append(re.sub(r"\.LBB\d+_\d+", ".LBB", ins))
    names = subprocess.run(["c++filt"], input="\n".join(kernels), capture_output=True, text=True).stdout.split("\n")
    res = {dm: kernels[k] for k, dm in zip(kernels, names) if kernels[k] and "(" in dm}
    json.dump(res, open(out, "w"))
    print(f"{len(res)} kernels -> {out}")


def diff(a, b, maps):
    A, B = json.load(open(a)), json.load(open(b))
    sub = [(m[0], m[1].split("=", 1)) for m in maps]

    def key(n):
        for kind, (old, new) in sub:
            n = re.sub(old, new, n) if kind == "re" else n.replace(old, new)
        return n
    Am = {key(n): v for n, v in A.items()}
    same, differ, missing = [], [], []
    for n, v in Am.items():
        if n not in B:
            missing.append(n)
        elif B[n] == v:
            same.append(n)
        else:
            differ.append(n)
    for n in same:
        print("identical ", n)
    for n in differ:
        print("DIFFERENT ", n, len(Am[n]), len(B[n]))
    for n in missing:
        print("unmatched ", n)
    print(f"{len(same)} identical, {len(differ)} different, {len(missing)} unmatched of {len(Am)} before; "
          f"{len(B)} kernels after")
    return 1 if differ else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2], sys.argv[3])
    else:
        maps = [(x[2:], sys.argv[i + 1]) for i, x in enumerate(sys.argv) if x in ("--map", "--re")]
        sys.exit(diff(sys.argv[2], sys.argv[3], maps))
