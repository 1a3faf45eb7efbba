"""Build the pybind11 `_C` stub that INTEGRATION.md section 3 documents (the compiled route
a maintainer would add next to the reference's DGR/ext.cpp:15-19), straight from the
markdown, against libgsr.so.  Test infrastructure: tests/test_stub_ext.py imports it and
__graft_entry__.build() builds it beforehand (the GPU box only loads the prebuilt module).

The block is compiled with the host compiler through torch.utils.cpp_extension with
with_cuda=False (no hipify pass: the stub is written against HIP's headers directly), the
ROCm include path, HIP platform define and the torch_hip / c10_hip / amdhip64 libraries."""
import hashlib
import importlib.util
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd", "diff_gaussian_rasterization")
BUILD = os.path.join(ROOT, "build", "ext_gsr")
NAME = "ext_gsr_stub"


def stub_source():
    """The ```cpp block of INTEGRATION.md that starts with `// ext_gsr.cpp`."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"```cpp\n(// ext_gsr\.cpp.*?)```", text, re.S)
    if not m:
        raise RuntimeError("INTEGRATION.md has no `// ext_gsr.cpp` code block")
    return m.group(1)


def so_path():
    return os.path.join(BUILD, NAME + ".so")


def build(verbose=False):
    """Compile the stub into build/ext_gsr/ (rebuilt when the markdown block or gsr.h changes)."""
    import torch.utils.cpp_extension as ce
    os.makedirs(BUILD, exist_ok=True)
    src = stub_source()
    cpp = os.path.join(BUILD, "ext_gsr.cpp")
    if not os.path.exists(cpp) or open(cpp).read() != src:
        with open(cpp, "w") as f:
            f.write(src)
    ce.load(name=NAME, sources=[cpp], build_directory=BUILD, with_cuda=False, verbose=verbose,
            extra_include_paths=[os.path.join(ROOT, "include"), "/opt/rocm/include"],
            extra_cflags=["-O1", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"],
            extra_ldflags=["-L" + LIBDIR, "-lgsr", "-Wl,-rpath," + LIBDIR, "-L/opt/rocm/lib", "-lamdhip64",
                           "-lc10_hip", "-ltorch_hip"])
    return so_path()


def load():
    """The prebuilt module (fails loudly when build() has not run)."""
    import torch  # noqa: F401  (the module links torch's libraries)
    path = so_path()
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run __graft_entry__.build() (or tests/stub_ext.py) first")
    spec = importlib.util.spec_from_file_location(NAME, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def source_digest():
    return hashlib.sha256(stub_source().encode()).hexdigest()[:16]


if __name__ == "__main__":
    print(build(verbose=True))
