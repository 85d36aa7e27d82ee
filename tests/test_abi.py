"""The C-ABI boundary: libftar.so builds, loads, and exports exactly include/ftar.h.

No compute calls here (no GPU in the CPU suite); the product must fail loudly without a
device instead of falling back to the CPU.
"""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fault-tolerant_amd", "lib", "libftar.so")
HEADER = os.path.join(ROOT, "include", "ftar.h")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "fault-tolerant_amd"), "-j8"], check=True)
    return LIB


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(ftar_\w+)\s*\(", src, flags=re.M))
    return names


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_header_declares_the_boundary():
    names = declared_functions()
    for fn in ("ftar_init", "ftar_allreduce_rabenseifner", "ftar_recursive_doubling", "ftar_reduce_local",
               "ftar_finalize", "ftar_abort", "ftar_barrier"):
        assert fn in names
    assert len(names) >= 20


def test_exports_exactly_the_header(built):
    assert exported_symbols(built) == declared_functions()


def test_library_loads_and_binds(built):
    L = ctypes.CDLL(built)
    for name in declared_functions():
        assert hasattr(L, name)
    L.ftar_version.restype = ctypes.c_char_p
    assert b"gfx950" in L.ftar_version()


def test_kernels_are_gfx950_code_objects(built, tmp_path):
    """The HIP kernels are compiled for gfx950 and nothing else (no CUDA/dual path).
    (llvm-objdump --offloading extracts the images next to its input: a copy in tmp_path,
    so nothing lands in lib/.)"""
    import shutil
    copy = str(tmp_path / "libftar.so")
    shutil.copy(built, copy)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", copy], capture_output=True,
                         text=True).stdout
    assert "gfx950" in out
    for other in ("gfx90a", "gfx942", "sm_"):
        assert other not in out


def test_init_fails_loudly_without_gpu(built):
    """No GPU here: ftar_init must return an error (no CPU fallback, no hang)."""
    code = (
        "import ctypes,sys\n"
        f"L=ctypes.CDLL({built!r})\n"
        "h=ctypes.c_void_p()\n"
        "rc=L.ftar_init(ctypes.byref(h))\n"
        "sys.exit(0 if rc!=0 else 1)\n"
    )
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "FTAR_JOB"):
        env.pop(k, None)
    cp = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    if cp.returncode != 0:
        pytest.skip("a HIP device is visible here")  # only meaningful on the GPU-less box
    assert cp.returncode == 0


def test_python_binding_has_no_fallback(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import conftest
    mod = conftest.load_package()
    monkeypatch.setattr(mod, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(mod, "_lib", None)
    with pytest.raises(mod.FtarError):
        mod.lib()


def test_oracle_is_not_linked_into_the_product(built):
    out = subprocess.run(["ldd", built], capture_output=True, text=True).stdout
    assert "oracle" not in out
    assert not any("oracle" in s for s in exported_symbols(built))


def test_op_type_check_before_any_device_call(built):
    """MPI_Reduce_local's type/op rule at the boundary, before anything touches a GPU:
    a logical / bitwise op on a float type is MPI_ERR_OP (9), an unknown op or type is
    MPI_ERR_ARG (13); every op MPI defines for the integer types is accepted (an empty
    reduce returns success without a device)."""
    L = ctypes.CDLL(built)
    L.ftar_reduce_local.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p]
    for dt in (0, 2):  # int32, int64
        for op in range(10):
            assert L.ftar_reduce_local(None, None, 0, dt, op, None) == 0, (dt, op)
    for dt in (1, 3):  # float32, float64
        for op in range(4):
            assert L.ftar_reduce_local(None, None, 0, dt, op, None) == 0, (dt, op)
        for op in range(4, 10):
            assert L.ftar_reduce_local(None, None, 0, dt, op, None) == 9, (dt, op)
    assert L.ftar_reduce_local(None, None, 0, 0, 10, None) == 13
    assert L.ftar_reduce_local(None, None, 0, 4, 0, None) == 13


def test_python_structs_mirror_the_header(tmp_path):
    """The ctypes mirrors of the header's structs (fault-tolerant_amd/__init__.py: Stats, Kill)
    have the C layout field for field -- a field added on one side only would shift every
    later one silently.  Offsets and sizes from a C program compiled against include/ftar.h."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ftar_abi_mirror", os.path.join(ROOT, "fault-tolerant_amd",
                                                                                 "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    src = open(HEADER).read()
    checks = []
    for cls, cname in ((m.Stats, "ftar_stats"), (m.Kill, "ftar_kill")):
        body = re.search(r"typedef struct\s*\{([^{}]*)\}\s*" + cname + r"\s*;", re.sub(r"/\*.*?\*/", "", src, flags=re.S))
        assert body, cname
        cfields = re.findall(r"(\w+)\s*;", body.group(1))
        assert [f for f, _ in cls._fields_] == cfields, (cname, cfields)
        checks.append((cls, cname, cfields))
    prog = tmp_path / "layout.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ftar.h"', "int main(void) {"]
    for _, cname, cfields in checks:
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        lines += [f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));' for f in cfields]
    lines.append("return 0; }")
    prog.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                       check=True).stdout.splitlines())
    for cls, cname, cfields in checks:
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f in cfields:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_test_hooks_are_not_in_the_product(built):
    """The test-only switches (FTAR_TRACE_DROP: a drain without its release; FTAR_KILL_WITHDRAW:
    a dying rank rewrites the control block) are compiled only into the TEST-ONLY hooks build
    (lib/libftar_hooks.so, -DFTAR_TEST_HOOKS) that the GPU tests needing them load; the product
    library does not contain them, and both export the same C ABI."""
    hooks = os.path.join(ROOT, "fault-tolerant_amd", "lib", "libftar_hooks.so")
    prod = open(built, "rb").read()
    for name in (b"FTAR_TRACE_DROP", b"FTAR_KILL_WITHDRAW", b"FTAR_PEER_WAIT_DELAY_US", b"FTAR_FAIL_IMPORT"):
        assert name not in prod, name
        assert name in open(hooks, "rb").read(), name
    assert exported_symbols(hooks) == exported_symbols(built) == declared_functions()


def _tree_src_id():
    return subprocess.run([os.path.join(ROOT, "fault-tolerant_amd", "tools", "build_id.sh"), "src"],
                          capture_output=True, text=True, check=True).stdout.strip()


def test_library_is_built_from_this_tree(built):
    """ftar_build_id() carries the digest of every product source the library was linked from:
    after make it is the digest of the tree's sources, so a result of this library is a result
    of this tree."""
    L = ctypes.CDLL(built)
    L.ftar_build_id.restype = ctypes.c_char_p
    got = L.ftar_build_id().decode()
    assert re.fullmatch(r"ftar-build abi=[0-9a-f]{16} src=[0-9a-f]{16}", got), got
    assert got.endswith("src=" + _tree_src_id())


def test_stale_launcher_is_refused(hostsim, tmp_path):
    """A launcher built from other headers than the library (a stale ftrun next to a new
    libftar): the rank refuses to attach with one line naming both builds, and the job ends
    instead of running with mismatched control-block layouts."""
    pkg = os.path.join(ROOT, "fault-tolerant_amd")
    stale = tmp_path / "ftrun_stale"
    subprocess.run(["gcc", "-O1", "-std=c11", "-D_GNU_SOURCE", "-DFTAR_ABI_ID=0x1234abcdull", "-o", str(stale),
                    os.path.join(pkg, "tools", "ftrun.c"), os.path.join(pkg, "csrc", "ftar_ctrl.c"),
                    "-lpthread", "-lrt"], check=True)
    env = dict(os.environ, FTAR_HOSTSIM_TAG=f"stale{os.getpid()}", FTAR_PROBE_DIR=str(tmp_path),
               FTAR_PROBE_ALGO="raben", FTAR_PROBE_COUNT="16", FTAR_PROBE_DTYPE="0")
    cp = subprocess.run([str(stale), "-np", "2", os.path.join(hostsim, "bin", "ftar_probe")], env=env,
                        capture_output=True, text=True, timeout=60)
    assert cp.returncode != 0
    assert "created by build 000000001234abcd" in cp.stderr and "different builds" in cp.stderr, cp.stderr[-1500:]
