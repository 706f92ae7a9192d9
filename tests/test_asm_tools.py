"""tools/asm_audit.py and tools/kinfo.py on small hand-written assembly (CPU): the audit flags a
compiler instruction that names an asm load's destination before its counted wait, and an asm
16-byte store without s_nop; kinfo counts the compiler's vmcnt waits and skips asm ones
(the vmcnt(0) drains)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
import asm_audit  # noqa: E402
import kinfo  # noqa: E402

HEAD = "_ZN3fooEv:\n"
TAIL = "\t.size\t_ZN3fooEv, 4\n"


def _write(tmp_path, body):
    p = tmp_path / "k.s"
    p.write_text(HEAD + body + TAIL)
    return str(p)


def test_audit_flags_early_use_of_asm_load(tmp_path):
    body = ("\t;;#ASMSTART\n\tds_read_b64_tr_b16 v[4:5], v1 offset:0\n\t;;#ASMEND\n"
            "\tv_mov_b32_e32 v9, v5\n"
            "\t;;#ASMSTART\n\ts_waitcnt lgkmcnt(0)\n\t;;#ASMEND\n")
    assert asm_audit.audit(_write(tmp_path, body)) == 1


def test_audit_accepts_use_after_wait(tmp_path):
    body = ("\t;;#ASMSTART\n\tglobal_load_dwordx4 v[4:7], v[0:1], off\n\t;;#ASMEND\n"
            "\tv_add_u32_e32 v9, v10, v11\n"
            "\t;;#ASMSTART\n\ts_waitcnt vmcnt(0)\n\t;;#ASMEND\n"
            "\tv_mov_b32_e32 v9, v5\n"
            "\t;;#ASMSTART\n\tglobal_store_dwordx4 v[0:1], v[4:7], off nt\n\ts_nop 1\n\t;;#ASMEND\n")
    assert asm_audit.audit(_write(tmp_path, body)) == 0


def test_audit_flags_store_without_nop(tmp_path):
    body = "\t;;#ASMSTART\n\tglobal_store_dwordx4 v[0:1], v[4:7], off nt\n\t;;#ASMEND\n"
    assert asm_audit.audit(_write(tmp_path, body)) == 1


def test_kinfo_counts_compiler_waits_only(tmp_path, capsys):
    body = ("\ts_waitcnt vmcnt(0)\n\tv_mfma_f32_32x32x16_f16 a[0:15], v[0:3], v[4:7], a[0:15]\n"
            "\t;;#ASMSTART\n\ts_waitcnt vmcnt(0)\n\t;;#ASMEND\n\ts_barrier\n\tscratch_load_dword v1, off, off\n")
    kinfo.main(_write(tmp_path, body), "foo")
    out = capsys.readouterr().out
    assert "scratch 1 mfma 1 barrier 1" in out and "'s_waitcnt vmcnt(0)': 1" in out


def test_audit_counts_outstanding_ops_per_counter(tmp_path):
    """vmcnt(N) retires all but the N youngest vector-memory operations: after two asm
    loads and vmcnt(1) the older one has landed and the younger may not have."""
    body = ("\t;;#ASMSTART\n\tglobal_load_dwordx4 v[4:7], v[0:1], off\n\t;;#ASMEND\n"
            "\t;;#ASMSTART\n\tglobal_load_dwordx4 v[8:11], v[2:3], off\n\t;;#ASMEND\n"
            "\t;;#ASMSTART\n\ts_waitcnt vmcnt(1)\n\t;;#ASMEND\n"
            "\tv_mov_b32_e32 v20, v4\n"     # older load: retired
            "\tv_mov_b32_e32 v21, v8\n")    # younger load: may be in flight
    assert asm_audit.audit(_write(tmp_path, body)) == 1


def test_audit_counts_compiler_memory_ops(tmp_path):
    """A compiler store issued after the asm load is one of the N youngest: vmcnt(1) then covers
    the asm load (it is older than the store)."""
    body = ("\t;;#ASMSTART\n\tglobal_load_dwordx4 v[4:7], v[0:1], off\n\t;;#ASMEND\n"
            "\tglobal_store_dword v[0:1], v9, off\n"
            "\ts_waitcnt vmcnt(1)\n"
            "\tv_mov_b32_e32 v20, v4\n")
    assert asm_audit.audit(_write(tmp_path, body)) == 0


def test_audit_scalar_loads_are_out_of_order(tmp_path):
    """A scalar load outstanding: lgkmcnt(1) retires nothing for certain."""
    body = ("\t;;#ASMSTART\n\tds_read_b64_tr_b16 v[4:5], v1 offset:0\n\t;;#ASMEND\n"
            "\ts_load_dword s4, s[0:1], 0x0\n"
            "\ts_waitcnt lgkmcnt(1)\n"
            "\tv_mov_b32_e32 v9, v5\n")
    assert asm_audit.audit(_write(tmp_path, body)) == 1


def test_build_audits_its_device_assembly():
    """build() keeps every file's device assembly (-save-temps=obj) and runs the audit over it;
    on the product build directory it finds nothing (skipped where the library was not built
    in this checkout)."""
    import pytest
    from mli_nerf_amd import build as b
    d = os.path.join(b.CSRC, "build")
    s_files = [f for f in os.listdir(d) if f.endswith("gfx950.s")] if os.path.isdir(d) else []
    if len(s_files) < len(b.SOURCES):
        pytest.skip("the library was not built in this checkout")
    assert b.audit_asm(d) == []
