"""CPU-side checks of the C-ABI library: it loads, exports every symbol the header declares, and the
ctypes mirrors of the argument structs have the C layout (no GPU needed, no compute calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "kwhisper.h")
LIB = os.path.join(ROOT, "kotoba-whisper_amd", "kwhisper", "libkwhisper.so")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kw_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "kotoba-whisper_amd", "csrc"), "-j8"], check=True)
    from kwhisper import _lib

    return _lib.load()


def test_exports_every_declared_symbol(lib):
    names = _declared()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    from kwhisper import _lib

    assert set(names) == set(_lib.EXPORTS), "ctypes binding and header disagree"


def test_version(lib):
    """The library's version equals the one include/kwhisper.h documents (INTEGRATION.md reads it the same way)."""
    import re

    with open(os.path.join(ROOT, "include", "kwhisper.h")) as f:
        want = int(re.search(r"int kw_version\(void\);\s*/\*\s*(\d+)\s*\*/", f.read()).group(1))
    assert lib.kw_version() == want == 112


def _c_layout(struct, fields):
    code = "#include <stdio.h>\n#include <stddef.h>\n#include \"kwhisper.h\"\nint main(){"
    code += f'printf("%zu\\n", sizeof({struct}));'
    for f in fields:
        code += f'printf("%zu\\n", offsetof({struct}, {f}));'
    code += "return 0;}"
    d = os.environ.get("TMPDIR", "/tmp")
    src, exe = os.path.join(d, "kw_layout.c"), os.path.join(d, "kw_layout")
    open(src, "w").write(code)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
    return [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]


@pytest.mark.parametrize("cname,pyname", [("kw_gemm_args", "GemmArgs"), ("kw_sampler_args", "SamplerArgs"),
                                          ("kw_dec_linear_args", "DecLinearArgs"),
                                          ("kw_dec_qkv_self_args", "QkvSelfArgs"),
                                          ("kw_dec_xq_cross_args", "XqCrossArgs")])
def test_struct_layout_matches_c(cname, pyname):
    from kwhisper import _lib

    cls = getattr(_lib, pyname)
    fields = [f for f, _ in cls._fields_]
    got = _c_layout(cname, fields)
    assert got[0] == ctypes.sizeof(cls)
    for f, off in zip(fields, got[1:]):
        assert getattr(cls, f).offset == off, f


def test_errors_are_returned_not_thrown(lib):
    """Invalid arguments come back as KW_EINVAL with a message (no HIP call is made)."""
    rc = lib.kw_layernorm(None, 1, 7, None, None, 1e-5, None, 0, None, None)
    assert rc == 1
    assert b"kw_layernorm" in lib.kw_last_error()


def test_torch_ops_register_every_entry_point(lib):
    """torch.ops.kw (libkwhisper_torch.so) loads beside the C ABI and registers one operator per
    launching entry point, each mutating its outputs in place (schema annotations) with a CUDA (HIP) kernel."""
    import torch

    from kwhisper import _lib

    kw = _lib.load_torch_ops()
    assert int(kw.version()) == lib.kw_version()
    for name in _lib.TORCH_OPS:
        schema = str(getattr(kw, name).default._schema)
        assert schema.startswith(f"kw::{name}(") and schema.endswith("-> ()"), schema
        assert "(a!)" in schema, schema
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"kw::{name}", "CUDA"), name
    assert int(kw.workspace_bytes("dec_linear", [1280, 5120])) == lib.kw_dec_linear_workspace_bytes(1280, 5120)
    # ABI symbols bound by the torch library are the header's (no private re-implementation)
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.TORCH_LIB_PATH], capture_output=True, text=True).stdout
    used = set(re.findall(r"\b(kw_[a-z0-9_]+)\b", out))
    assert used and used <= set(_declared()), used - set(_declared())


def test_torch_ops_reject_host_tensors(lib):
    """No CPU path: a host tensor is refused with ValueError before any launch."""
    import torch

    from kwhisper import _lib

    kw = _lib.load_torch_ops()
    with pytest.raises((ValueError, NotImplementedError)):
        kw.attention(torch.zeros(3 * 64), 1, 1, 1, 64, torch.zeros(64))


def test_integration_doc_names_only_declared_symbols():
    """every ``kw_*`` entry point INTEGRATION.md names (its ABI table, the ctypes stub) is one the
    header declares -- so a symbol that leaves the library cannot linger in the maintainer's guide.  Struct and type
    names (kw_*_args, kw_stream_t) are not entry points."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    named = {n for n in re.findall(r"\b(kw_[a-z0-9_]+)\b", doc) if not n.endswith(("_args", "_t"))}
    # "`kw_dec_qkv_self` (+ `_workspace`, `_supported`)": the suffixes name kw_dec_qkv_self_workspace etc.
    for base, rest in re.findall(r"`(kw_[a-z0-9_]+)` \(\+ ([^)]*)\)", doc):
        named |= {base + s for s in re.findall(r"`(_[a-z0-9_]+)`", rest)}
    missing = sorted(named - set(_declared()))
    assert named and not missing, missing
    # and the other way round: every entry point the header declares is in the guide
    undocumented = sorted(set(_declared()) - named)
    assert not undocumented, undocumented
