"""C-ABI library checks that need no GPU: the shared library loads, exports every entry
point include/dad.h declares, and the ctypes mirrors have the C layout."""
import ctypes
import os
import re
import subprocess

import pytest

import dadpkg

ROOT = dadpkg.ROOT
HEADER = os.path.join(ROOT, "include", "dad.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**(dad_[a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    p = dadpkg.pkg()
    p.build(verbose=False)
    L = p.lib()
    names = _declared_functions()
    assert len(names) >= 15, names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # the ctypes binding table covers exactly the header's entry points
    assert sorted(p._lib.EXPORTS) == names


def test_host_only_queries():
    p = dadpkg.pkg()
    L = p.lib()
    assert L.dad_param_count() == 256 * 768 + 256 + 4 * 256 + 4
    cfg = p.dad_config_for(p.ConfigView(flavor="iemocap"), 64, 300, 64, 300, 60, 1)
    n = ctypes.c_size_t(0)
    assert L.dad_workspace_bytes(cfg, ctypes.byref(n)) == 0
    assert n.value > 0
    bad = p.dad_config_for(p.ConfigView(flavor="iemocap"), 64, 300, 64, 300, 60, 1)
    bad.B = 0
    assert L.dad_workspace_bytes(bad, ctypes.byref(n)) == 1002       # DAD_E_SHAPE
    assert L.dad_error_string(1001).decode().startswith("DAD_E_ARG")
    assert L.dad_encoder_workspace_bytes(8, 20) > 0


@pytest.mark.parametrize("Bc,Tc,Bn,Tn,cus", [
    (64, 300, 64, 300, 256),       # the bench geometry
    (1024, 300, 1024, 1280, 256),  # long noisy batch: strong jobs hold 2.0 live sub-slabs, clean ones 1.9
    (1024, 1280, 1024, 300, 256),
    (1024, 2000, 1024, 30, 8),     # few CUs: many jobs per workgroup on both sides
    (1000, 40, 3, 4000, 4),
])
def test_encoder_ws_plan_keeps_every_range_within_the_kernel_table(Bc, Tc, Bn, Tn, cus):
    """The BF16 encoder's job table holds DAD_ENC_WS_MAXJ = 256 jobs per workgroup.  The host
    plan (the kernel's own range function, priced in live sub-slabs) must never exceed it,
    including geometries where clean and strong jobs hold different numbers of sub-slabs."""
    p = dadpkg.pkg()
    L = p.lib()
    for epoch in (0, 60):
        cfg = p.dad_config_for(p.ConfigView(flavor="iemocap"), Bc, Tc, Bn, Tn, epoch, 1,
                               precision=p._lib.PREC_BF16)
        nt, ns, mj = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        assert L.dad_encoder_ws_plan(cfg, cus, ctypes.byref(nt), ctypes.byref(ns), ctypes.byref(mj)) == 0
        assert 0 < mj.value <= 256, (Bc, Tc, Bn, Tn, cus, epoch, nt.value, ns.value, mj.value)
        assert ns.value >= 1 and (nt.value >= 1) == (epoch >= 30)


@pytest.mark.parametrize("Bc,Tc,Bn,Tn,cus", [
    (64, 300, 64, 300, 256),       # the bench geometry
    (64, 300, 48, 250, 256),       # Bc != Bn, Tc != Tn
    (7, 20, 5, 33, 256),           # fewer slabs than CUs
    (1024, 300, 1024, 1280, 256),  # long noisy batch
    (64, 300, 64, 300, 304),       # a CU count that is not 256
    (64, 300, 64, 300, 252),       # CUs not divisible by 8
])
def test_encoder_job_assignment_covers_every_slab_once(Bc, Tc, Bn, Tn, cus):
    """Every clean, weak and strong 32-row slab is run by exactly one workgroup of the prepared-row
    encoder in the right role (teachers: weak slabs; students: clean slabs j < Jc, strong slabs
    Jc + s), and no workgroup's range exceeds the kernel's 256-job table."""
    p = dadpkg.pkg()
    L = p.lib()
    for epoch in (0, 60):
        cfg = p.dad_config_for(p.ConfigView(flavor="iemocap"), Bc, Tc, Bn, Tn, epoch, 1,
                               precision=p._lib.PREC_FP16)
        nt, ns, mj = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert L.dad_encoder_ws_plan(cfg, cus, ctypes.byref(nt), ctypes.byref(ns), ctypes.byref(mj)) == 0
        need = 4 * (nt.value + ns.value)
        if need > 4 * cus:     # the grid outgrew cus: a 4*cus table is refused, nothing written
            small = (ctypes.c_int * (4 * cus))(*([-7] * (4 * cus)))
            assert L.dad_encoder_ws_jobs(cfg, cus, small, 4 * cus) == 1001
            assert all(v == -7 for v in small)
        assert L.dad_encoder_ws_jobs(cfg, cus, (ctypes.c_int * (need - 1))(), need - 1) == 1001
        buf = (ctypes.c_int * need)()
        grid = L.dad_encoder_ws_jobs(cfg, cus, buf, need)
        assert grid == nt.value + ns.value > 0
        ncc, ncn = -(-Tc // 32), -(-Tn // 32)
        Jc, Js = Bc * ncc, (Bn * ncn if epoch >= 30 else 0)
        seen_t, seen_s = {}, {}
        for wg in range(grid):
            t, a0, st, nj = buf[4 * wg:4 * wg + 4]
            assert 0 <= nj <= 256 and st >= 1
            for j in range(a0, a0 + nj * st, st):
                d = seen_t if t else seen_s
                assert j not in d, (wg, j)
                d[j] = wg
        assert sorted(seen_t) == list(range(Js))
        assert sorted(seen_s) == list(range(Jc + Js))


def test_ctypes_structs_match_c_layout(tmp_path):
    """Compile a C probe against include/dad.h and compare sizeof/offsetof with ctypes."""
    p = dadpkg.pkg()
    fields = {"dad_config": p._lib.DadConfig, "dad_batch": p._lib.DadBatch, "dad_state": p._lib.DadState}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "dad.h"', "int main(void){"]
    for cname, cls in fields.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in cls._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f[0], cname, f[0]))
    lines.append("return 0;}")
    c = tmp_path / "probe.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)])
    out = dict(l.split() for l in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, cls in fields.items():
        assert int(out[cname]) == ctypes.sizeof(cls), cname
        for f in cls._fields_:
            assert int(out["%s.%s" % (cname, f[0])]) == getattr(cls, f[0]).offset, (cname, f[0])


def test_no_oracle_import_in_product():
    pkgdir = os.path.join(ROOT, dadpkg.PKG_NAME)
    for dp, _, fs in os.walk(pkgdir):
        for f in fs:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle" not in re.findall(r"(?:import|from)\s+(oracle)\b", txt), f
                assert "/root/reference" not in txt, f


def test_abi_version_checked_at_load(monkeypatch):
    """the library reports the ABI it was built for and the binding refuses a stale build
    at load (here: a binding that expects another version)."""
    p = dadpkg.pkg()
    L = p.lib()
    assert L.dad_abi_version() == p._lib.DAD_ABI_VERSION
    hdr = open(HEADER).read()
    assert "#define DAD_ABI_VERSION %d" % p._lib.DAD_ABI_VERSION in hdr
    monkeypatch.setattr(p._lib, "_LIB", None)
    monkeypatch.setattr(p._lib, "DAD_ABI_VERSION", p._lib.DAD_ABI_VERSION + 1)
    with pytest.raises(p._lib.DadError, match="rebuild"):
        p._lib.lib()
