"""The committed Rust FFI shim (integration/rust/src/hip/mod.rs, the drop-in for
src/cuda/mod.rs:337-450) against the C-ABI it binds (include/rrt_hip.h).

There is no Rust toolchain in this image, so the shim cannot be compiled here; instead every
`extern "C"` declaration is parsed and checked against the header's prototype (name, argument
count, order and types, return type), every `#[repr(C)]` mirror struct against the header's
field list, the shim's constants against the header's #defines, and every bound symbol against
librrt_hip.so's dynamic exports when the library is built. main_rs.patch must be a well-formed
unified diff that adds `mod hip;` and the `--backend hip` arm next to the CUDA one.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "integration", "rust", "src", "hip", "mod.rs")
HEADER = os.path.join(ROOT, "include", "rrt_hip.h")
LIB = os.path.join(ROOT, "rustraytrace_amd", "librrt_hip.so")

# Rust type in the shim -> C type in the header. The reference's #[repr(C)] scene structs
# (gpu/mod.rs:13-42) are byte-identical to the header's (tests/test_abi.py).
RUST_TO_C = {
    "*const CameraUniform": "const RrtCamera *",
    "*const SphereGpu": "const RrtSphere *",
    "*const MaterialGpu": "const RrtMaterial *",
    "*const RrtTexture": "const RrtTexture *",
    "*const RrtSceneExt": "const RrtSceneExt *",
    "u32": "uint32_t",
    "i32": "int32_t",
    "u64": "uint64_t",
    "usize": "size_t",
    "f32": "float",
    "*mut f32": "float *",
    "*const f32": "const float *",
    "*mut f64": "double *",
    "*const f64": "const double *",
    "*mut u8": "uint8_t *",
    "*const u8": "const uint8_t *",
    "*mut i32": "int32_t *",
    "*const c_char": "const char *",
    "*mut c_void": "void *",
}


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", " ", s, flags=re.S)


def _strip_rust_comments(s):
    return re.sub(r"//[^\n]*", " ", s)


def _norm_c_type(t):
    t = re.sub(r"\s+", " ", t.replace("*", " * ")).strip()
    return t.replace(" *", " *").replace("* ", "* ").replace(" * ", " *").replace("  ", " ").strip()


def _c_param_type(p):
    p = re.sub(r"\s+", " ", p).strip()
    m = re.match(r"^(.*?)(\w+)$", p)  # drop the parameter name
    assert m, p
    return _norm_c_type(m.group(1))


def header_prototypes():
    src = _strip_c_comments(open(HEADER).read())
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w \*]*?)\b(rrt_\w+)\s*\(([^()]*)\)\s*;", src):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        if name in protos:
            continue
        args = [] if params in ("", "void") else [_c_param_type(p) for p in params.split(",")]
        protos[name] = (_norm_c_type(ret), args)
    return protos


def header_struct(name):
    src = _strip_c_comments(open(HEADER).read())
    m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, flags=re.S)
    assert m, name
    fields = []
    for decl in m.group(1).split(";"):
        decl = re.sub(r"\s+", " ", decl).strip()
        if decl:
            fields.append((decl.rsplit(" ", 1)[-1].lstrip("*"), _c_param_type(decl)))
    return fields


def shim_externs():
    src = _strip_rust_comments(open(SHIM).read())
    block = re.search(r'extern "C" \{(.*?)\n    \}', src, flags=re.S)
    assert block, "no extern \"C\" block in the shim"
    out = {}
    for m in re.finditer(r"fn (\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block.group(1), flags=re.S):
        name, params, ret = m.group(1), m.group(2), (m.group(3) or "()").strip()
        args = []
        for p in [p for p in params.split(",") if p.strip()]:
            pname, ptype = p.split(":", 1)
            args.append((pname.strip(), re.sub(r"\s+", " ", ptype).strip()))
        out[name] = (ret, args)
    return out


def shim_struct(name):
    src = _strip_rust_comments(open(SHIM).read())
    m = re.search(r"pub struct %s \{(.*?)\}" % name, src, flags=re.S)
    assert m, name
    fields = []
    for line in m.group(1).split(","):
        line = line.strip()
        if line:
            fname, ftype = line.replace("pub ", "").split(":", 1)
            fields.append((fname.strip(), re.sub(r"\s+", " ", ftype).strip()))
    return fields


def test_shim_files_present():
    for rel in ["src/hip/mod.rs", "build.rs", "Cargo.toml.fragment", "main_rs.patch"]:
        assert os.path.isfile(os.path.join(ROOT, "integration", "rust", rel)), rel


def test_every_extern_matches_the_header():
    protos = header_prototypes()
    externs = shim_externs()
    assert {"rrt_hip_render", "rrt_hip_render_ex", "rrt_hip_last_error", "rrt_hip_abi_version"} <= set(externs)
    for name, (ret, args) in externs.items():
        assert name in protos, f"{name} is bound by the shim but not declared in rrt_hip.h"
        c_ret, c_args = protos[name]
        assert RUST_TO_C.get(ret, ret) == c_ret, (name, ret, c_ret)
        assert len(args) == len(c_args), (name, len(args), len(c_args))
        for i, ((pname, ptype), ctype) in enumerate(zip(args, c_args)):
            assert ptype in RUST_TO_C, f"{name} arg {i} ({pname}): unmapped Rust type {ptype}"
            assert RUST_TO_C[ptype] == ctype, f"{name} arg {i} ({pname}): {ptype} vs C {ctype}"


def test_header_parser_sees_the_drop_in_entry():
    # guards the checker itself: the drop-in entry has 11 parameters in this order
    ret, args = header_prototypes()["rrt_hip_render"]
    assert ret == "int32_t" and args == [
        "const RrtCamera *", "const RrtSphere *", "uint32_t", "const RrtMaterial *", "uint32_t",
        "const RrtTexture *", "uint32_t", "uint32_t", "uint32_t", "uint32_t", "float *"]
    assert header_prototypes()["rrt_hip_last_error"] == ("const char *", [])


@pytest.mark.parametrize("name", ["RrtTexture", "RrtSceneExt"])
def test_repr_c_mirrors_match_header_structs(name):
    c_fields = header_struct(name)
    r_fields = shim_struct(name)
    assert [f for f, _ in r_fields] == [f for f, _ in c_fields]
    for (fname, rtype), (_, ctype) in zip(r_fields, c_fields):
        if rtype == "*const c_void":  # opaque element pointer: any const pointer in C
            assert ctype.startswith("const ") and ctype.endswith("*"), (fname, ctype)
        else:
            assert RUST_TO_C.get(rtype) == ctype, (fname, rtype, ctype)


def test_shim_constants_match_header():
    src = open(SHIM).read()
    hdr = open(HEADER).read()
    abi = int(re.search(r"RRT_ABI_VERSION: u32 = (\d+);", src).group(1))
    assert abi == int(re.search(r"#define RRT_ABI_VERSION (\d+)u", hdr).group(1))
    quiet = int(re.search(r"RRT_FLAG_QUIET: u32 = (0x[0-9a-fA-F]+);", src).group(1), 16)
    assert quiet == int(re.search(r"#define RRT_FLAG_QUIET (0x[0-9a-fA-F]+)u", hdr).group(1), 16)


def test_bound_symbols_are_exported():
    if not os.path.exists(LIB):
        pytest.skip("librrt_hip.so not built")
    nm = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    missing = set(shim_externs()) - exported
    assert not missing, missing


def test_build_rs_links_only_with_the_feature():
    src = open(os.path.join(ROOT, "integration", "rust", "build.rs")).read()
    assert "CARGO_FEATURE_HIP" in src and "rustc-link-lib=dylib=rrt_hip" in src
    frag = open(os.path.join(ROOT, "integration", "rust", "Cargo.toml.fragment")).read()
    assert re.search(r"^hip = \[\]$", frag, flags=re.M)
    shim = open(SHIM).read()
    # both feature arms exist, like cuda/mod.rs:442-450
    assert '#[cfg(feature = "hip")]\npub fn render_in_one_weekend' in shim
    assert '#[cfg(not(feature = "hip"))]\npub fn render_in_one_weekend' in shim


def test_main_rs_patch_is_a_unified_diff_adding_the_hip_arm():
    patch = open(os.path.join(ROOT, "integration", "rust", "main_rs.patch")).read()
    lines = patch.splitlines()
    assert lines[0] == "--- a/src/main.rs" and lines[1] == "+++ b/src/main.rs"
    added = [ln[1:] for ln in lines if ln.startswith("+") and not ln.startswith("+++")]
    assert "mod hip;" in added
    assert any("hip::render_in_one_weekend()" in ln for ln in added)
    # hunk headers agree with their bodies (old/new line counts)
    i = 2
    while i < len(lines):
        m = re.match(r"@@ -(\d+),(\d+) \+(\d+),(\d+) @@", lines[i])
        assert m, lines[i]
        old_n, new_n = int(m.group(2)), int(m.group(4))
        j, o, n = i + 1, 0, 0
        while j < len(lines) and not lines[j].startswith("@@"):
            c = lines[j][:1]
            o += c in (" ", "-")
            n += c in (" ", "+")
            j += 1
        assert (o, n) == (old_n, new_n), lines[i]
        i = j
