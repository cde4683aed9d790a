"""CPU: libmccs_hip.so loads and exports every symbol include/*.h declares.

No compute calls here (no GPU in the build container).
"""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mccs_amd", "libmccs_hip.so")


def declared_functions():
    names = set()
    for h in ("mccs_hip.h",):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*[A-Za-z_][\w \*]*?\b(mccs\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def declared_kernels():
    """Reference-named kernel host stubs the header promises (symbol-level swap)."""
    src = open(os.path.join(ROOT, "include", "mccs_kernels.h")).read()
    return set(re.findall(r"^MCCS_KERNEL_SYMBOL\((\w+)\);", src, flags=re.M))


def exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_library_loads(lib):
    assert lib.mccs_hip_version().startswith(b"mccs_amd")


def test_every_declared_function_is_exported():
    decl = declared_functions()
    assert len(decl) >= 4
    missing = decl - exported()
    assert not missing, f"declared but not exported: {sorted(missing)}"


def test_every_declared_symbol_has_ctypes_signature():
    from mccs_amd import _lib

    missing = declared_functions() - set(_lib.SIGNATURES)
    assert not missing, sorted(missing)


def test_reference_kernel_symbols_exported():
    syms = exported()
    assert len(declared_kernels()) == 41  # 4 ops x 10 types + AllGather (collectives.h:43-49)
    for k in declared_kernels():
        assert k in syms, k


def test_code_object_targets_gfx950(tmp_path):
    fat = tmp_path / "fatbin.bin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fat)], check=True)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={fat}"], check=True, capture_output=True, text=True).stdout
    assert "hipv4-amdgcn-amd-amdhsa--gfx950" in out.split()
