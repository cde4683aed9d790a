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
    assert len(declared_kernels()) == 45  # 4 ops x 10 types + AllGather (collectives.h:43-49) + 4 ___nv_bfloat16
    for k in declared_kernels():
        assert k in syms, k


def test_code_object_targets_gfx950(tmp_path):
    fat = tmp_path / "fatbin.bin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fat)], check=True)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={fat}"], check=True, capture_output=True, text=True).stdout
    assert "hipv4-amdgcn-amd-amdhsa--gfx950" in out.split()


# A stub of the reference declarations (collectives.h:43-49 MCCS_KERN_NAME /
# DECL5 with C++ linkage, DECL2 type list with __nv_bfloat16), compiled with
# g++ so the compiler -- not this test -- mangles the names the reference's
# bindgen (-x c++) would bind.
REF_STUB = r"""
#include <stdint.h>
#include <stdio.h>
#include <dlfcn.h>
struct mccsDevComm;
struct mccsDevWork;
#define MCCS_KERN_NAME(func, algo, proto, devredop, type) mccsKernel_##func##_##algo##_##proto##_##devredop##_##type
#define DECL5(func, algo, proto, devredop, type) \
  extern void MCCS_KERN_NAME(func, algo, proto, devredop, type)(struct mccsDevComm* comm, uint64_t channelMask, \
                                                                struct mccsDevWork* workHead);
#define DECL3(func, devredop, type) DECL5(func, RING, SIMPLE, devredop, type)
#define DECL2(func, devredop) DECL3(func, devredop, int8_t) DECL3(func, devredop, uint8_t) \
  DECL3(func, devredop, int32_t) DECL3(func, devredop, uint32_t) DECL3(func, devredop, int64_t) \
  DECL3(func, devredop, uint64_t) DECL3(func, devredop, half) DECL3(func, devredop, float) \
  DECL3(func, devredop, double) DECL3(func, devredop, __nv_bfloat16)
DECL3(AllGather, Sum, int8_t)
DECL2(AllReduce, Sum) DECL2(AllReduce, Prod) DECL2(AllReduce, Min) DECL2(AllReduce, Max)
#define CHECK(name, cname) do { \
    void* c = dlsym(RTLD_DEFAULT, cname); \
    printf("%s %d\n", cname, c != 0 && c == (void*)&name); } while (0)
int main() {
  CHECK(mccsKernel_AllReduce_RING_SIMPLE_Sum_half, "mccsKernel_AllReduce_RING_SIMPLE_Sum_half");
  CHECK(mccsKernel_AllReduce_RING_SIMPLE_Prod_int32_t, "mccsKernel_AllReduce_RING_SIMPLE_Prod_int32_t");
  CHECK(mccsKernel_AllGather_RING_SIMPLE_Sum_int8_t, "mccsKernel_AllGather_RING_SIMPLE_Sum_int8_t");
  CHECK(mccsKernel_AllReduce_RING_SIMPLE_Sum___nv_bfloat16, "mccsKernel_AllReduce_RING_SIMPLE_Sum_bfloat16");
  CHECK(mccsKernel_AllReduce_RING_SIMPLE_Min_float, "mccsKernel_AllReduce_RING_SIMPLE_Min_float");
  return 0;
}
"""


def _ref_stub_names(tmp_path):
    src = tmp_path / "ref_decls.cpp"
    src.write_text(REF_STUB.split("#define CHECK")[0] + _address_table())
    obj = tmp_path / "ref_decls.o"
    subprocess.run(["g++", "-std=c++11", "-c", str(src), "-o", str(obj)], check=True)
    out = subprocess.run(["nm", "-u", str(obj)], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if "mccsKernel" in line}


def _address_table():
    # take every kernel's address so each declaration becomes an undefined reference
    names = ["mccsKernel_AllGather_RING_SIMPLE_Sum_int8_t"]
    for op in ("Sum", "Prod", "Min", "Max"):
        for t in ("int8_t", "uint8_t", "int32_t", "uint32_t", "int64_t", "uint64_t", "half", "float", "double",
                  "__nv_bfloat16"):
            names.append(f"mccsKernel_AllReduce_RING_SIMPLE_{op}_{t}")
    return "const void* table[] = {" + ", ".join(f"(const void*)&{n}" for n in names) + "};\n"


def test_reference_cxx_linkage_names_exported(tmp_path):
    """Every kernel the reference's collectives.h declares (C++ linkage, bf16
    as __nv_bfloat16) resolves in libmccs_hip.so, at the same address as the
    extern "C" handle (so hipLaunchKernel finds the registered kernel)."""
    want = _ref_stub_names(tmp_path)
    assert len(want) == 41 and all(w.startswith("_Z") for w in want), sorted(want)[:3]
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    addr = {line.split()[-1]: line.split()[0] for line in out.splitlines() if line.strip()}
    for m in want:
        assert m in addr, f"reference symbol {m} not exported"
        plain = m[2:].lstrip("0123456789").split("P11mccsDevComm")[0].replace("___nv_bfloat16", "_bfloat16")
        assert addr[m] == addr[plain], (m, plain)


def test_reference_declarations_link_and_resolve(tmp_path):
    """A C++ program written against the reference declarations links with
    libmccs_hip.so unchanged, and each name it takes the address of is the
    library's kernel handle."""
    src = tmp_path / "ref_link.cpp"
    src.write_text(REF_STUB)
    exe = tmp_path / "ref_link"
    lib_dir = os.path.dirname(LIB)
    subprocess.run(["g++", "-std=c++11", str(src), "-o", str(exe), f"-L{lib_dir}", "-lmccs_hip",
                    f"-Wl,-rpath,{lib_dir}", "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-ldl"], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    rows = [r.split() for r in out if r.strip()]
    assert len(rows) == 5 and all(r[1] == "1" for r in rows), rows
