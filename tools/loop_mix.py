#!/usr/bin/env python3
"""Instruction mix of the innermost loop(s) of GEMM kernels in libmvae_hip.so (gfx950 code objects).
    python3 tools/loop_mix.py <kernel-name-substring> [...]"""
import collections, os, re, subprocess, sys, tempfile

LLVM = "/opt/rocm/llvm/bin"
LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "medvae_disentangled_multimodal_amd", "libmvae_hip.so")


def code_objects(tmp):
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, os.path.join(tmp, "x")], check=True)
    d = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", d)]
    for i, o in enumerate(offs):
        b = os.path.join(tmp, f"b{i}")
        open(b, "wb").write(d[o:offs[i + 1] if i + 1 < len(offs) else len(d)])
        co = os.path.join(tmp, f"k{i}.co")
        if subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"]).returncode == 0:
            yield co


def main():
    pats = sys.argv[1:]
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(tmp):
            asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                                 text=True).stdout
            for blk in asm.split("\n\n"):
                m = re.search(r"<(\S+)>:", blk)
                if not m or not all(p in m.group(1) for p in pats):
                    continue
                ent = []
                for l in blk.splitlines():
                    mm = re.search(r"//\s*([0-9A-F]+):", l)
                    if mm:
                        ent.append((int(mm.group(1), 16), l.strip().split("//")[0].strip()))
                for k, (a, ins) in enumerate(ent):
                    mb = re.match(r"s_cbranch_\w+ (\d+)", ins)
                    if not mb:
                        continue
                    off = int(mb.group(1))
                    off = off - 65536 if off > 32767 else off
                    if off >= 0:
                        continue
                    tgt = a + 4 + off * 4
                    st = [n for n, (aa, _) in enumerate(ent) if aa == tgt]
                    if not st or k - st[0] > 2000:
                        continue
                    loop = [x for _, x in ent[st[0]:k + 1]]
                    c = collections.Counter(x.split()[0] for x in loop)
                    nm = sum(v for kk, v in c.items() if kk.startswith("v_mfma"))
                    if nm == 0:
                        continue
                    valu = sum(v for kk, v in c.items() if kk.startswith("v_") and not kk.startswith("v_mfma"))
                    print(f"{m.group(1)[:110]}\n  loop {len(loop)} instr: mfma {nm} valu {valu} "
                          f"ds_read {sum(v for kk, v in c.items() if kk.startswith('ds_read'))} "
                          f"ds_write {sum(v for kk, v in c.items() if kk.startswith('ds_write'))} "
                          f"vmem {sum(v for kk, v in c.items() if kk.startswith('buffer_'))} "
                          f"salu {sum(v for kk, v in c.items() if kk.startswith('s_'))}")
                    if os.environ.get("LOOP_DUMP"):  # per-opcode histogram, or the whole loop with LOOP_DUMP=asm
                        if os.environ["LOOP_DUMP"] == "asm":
                            print("\n".join(loop))
                        else:
                            print("  " + ", ".join(f"{kk} {v}" for kk, v in c.most_common()))
                    break


if __name__ == "__main__":
    main()
