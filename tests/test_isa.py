"""Machine-code checks of the built per-pair kernels (CPU only: they read the
gfx950 code objects the in-tree build leaves under word2vec_amd/lib/obj).

The LDS-private rows' per-row lock (w2v_kernels.hpp priv_lock / priv_unlock,
W2V_PRIV_ADD 2) is taken with a relaxed atomicOr and released with a relaxed
atomicAnd; its correctness rests on those, and the row's reads and writes
between them, being LDS instructions: one wave's LDS operations execute in
issue order, so the release cannot overtake the row's writes (a
generic pointer lowered to flat_* instructions would lose that ordering).
This asserts the lowering: the lock and mask atomics are ds_or_rtn_b32 /
ds_and_b32 / ds_or_b64 / ds_wrxchg_rtn_b64, and no flat atomic exists in the
kernels at all."""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
OBJ = ROOT / "word2vec_amd" / "lib" / "obj"
OBJDUMP = Path("/opt/rocm/lib/llvm/bin/llvm-objdump")


def _disasm(obj: Path, tmp: Path) -> str:
    dst = tmp / obj.name
    dst.write_bytes(obj.read_bytes())
    subprocess.run([str(OBJDUMP), "--offloading", str(dst)], check=True, capture_output=True, cwd=tmp)
    dev = [p for p in tmp.iterdir() if p.name.startswith(obj.name + ".") and "gfx950" in p.name]
    assert len(dev) == 1, dev
    return subprocess.run([str(OBJDUMP), "-d", str(dev[0])], check=True, capture_output=True, text=True).stdout


@pytest.mark.parametrize("nv", [2, 4, 5])
def test_private_row_lock_is_lds(nv, tmp_path):
    obj = OBJ / f"w2v_inst_nv{nv}.o"
    if not OBJDUMP.exists() or not obj.exists():
        pytest.skip("needs the in-tree build (word2vec_amd/csrc: make) and llvm-objdump")
    asm = _disasm(obj, tmp_path)
    ops = re.findall(r"\b(ds_or_rtn_b32|ds_and_b32|ds_or_b64|ds_wrxchg_rtn_b64|flat_atomic_\w+)\b", asm)
    assert ops.count("ds_or_rtn_b32") > 0 and ops.count("ds_and_b32") > 0  # lock taken / released in LDS
    assert ops.count("ds_or_rtn_b32") == ops.count("ds_and_b32")  # every acquire has its release
    assert ops.count("ds_or_b64") > 0  # the dirty masks
    assert [o for o in ops if o.startswith("flat_atomic")] == []
