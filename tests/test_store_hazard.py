"""Static guard for the gfx950 buffer-store hazard (GroupNorm at small per-sample sizes).

On gfx950 a VALU write to the data VGPRs of a just-issued multi-dword buffer store whose offset sits
in an SGPR `soffset` corrupts the store (the compiler inserts the required wait state only when
`soffset` is not a register; found with tools/gn_stress.py: ~1 % of the GroupNorm dx stores landed
wrong). Every multi-dword buffer store of the library must therefore carry its whole offset in the
VGPR and use the literal `soffset` 0. This test disassembles every gfx950 code object bundled in
libmvae_hip.so and fails on any `buffer_store_dwordx2/x3/x4` whose `soffset` operand is a register.
CPU only: llvm-objdump on the shipped binary, nothing runs on a GPU.
"""
import os
import re
import subprocess

import pytest

from medvae_disentangled_multimodal_amd import _lib

LLVM = "/opt/rocm/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
STORE = re.compile(r"\bbuffer_store_dwordx[234]\b(.*)")


def _code_objects(tmp_path):
    """The gfx950 code objects of the library: the .hip_fatbin section holds one offload bundle per
    linked translation unit (concatenated), each unbundled separately."""
    fat = tmp_path / "fat.bin"
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", _lib.LIB_PATH, str(tmp_path / "lib.tmp")],
                   check=True, capture_output=True)
    data = fat.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for i, o in enumerate(offs):
        end = offs[i + 1] if i + 1 < len(offs) else len(data)
        b = tmp_path / f"b{i}.bin"
        b.write_bytes(data[o:end])
        co = tmp_path / f"k{i}.co"
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                            f"--targets={TARGET}", f"--output={co}"], capture_output=True, text=True)
        if r.returncode == 0 and co.exists() and co.stat().st_size > 0:
            out.append(co)
    return out


def _soffset(operands: str) -> str:
    # operands: "vdata, vaddr, s[rsrc], soffset [offen] [offset:N] [nt ...]" (comment stripped)
    parts = [p.strip() for p in operands.split("//")[0].split(",")]
    return parts[3].split()[0] if len(parts) >= 4 else ""


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-objdump"), reason="ROCm llvm-objdump not installed")
def test_no_multidword_buffer_store_with_register_soffset(tmp_path):
    cos = _code_objects(tmp_path)
    assert cos, "no gfx950 code object found in libmvae_hip.so"
    n_stores, bad = 0, []
    for co in cos:
        asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(co)], check=True, capture_output=True,
                             text=True).stdout
        for line in asm.splitlines():
            m = STORE.search(line)
            if not m:
                continue
            n_stores += 1
            so = _soffset(m.group(1))
            if re.fullmatch(r"(s\d+|s\[\d+:\d+\]|ttmp\d+|m0|vcc_(lo|hi)|exec_(lo|hi))", so):
                bad.append(line.strip())
    # the GEMM / GroupNorm epilogues are all 16-B buffer stores: an empty scan means the parse broke
    assert n_stores > 1000, f"only {n_stores} multi-dword buffer stores parsed"
    assert not bad, f"{len(bad)} multi-dword buffer stores with a register soffset, e.g. {bad[:3]}"


def test_soffset_parser():
    assert _soffset(" v[4:7], v2, s[16:19], 0 offen") == "0"
    assert _soffset(" v[4:7], v2, s[16:19], s5 offen offset:16") == "s5"
