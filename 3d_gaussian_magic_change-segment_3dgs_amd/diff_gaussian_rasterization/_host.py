"""The compiled host binding (csrc/host_ext.cpp, torch extension "gsr_host"): the single-view
forward / backward host work of _C.py in C++ (argument checks, allocations, libgsr calls).

build() compiles it in-tree into build/ext_host/ (torch.utils.cpp_extension, host compiler, no
hipify pass; linked against libgsr.so); __graft_entry__.build() runs it.  load() returns the
prebuilt module, or None when it has not been built -- _C.py then does the same work over
ctypes (the same libgsr kernels; there is no CPU path either way).  GSR_HOST_EXT=0 forces the
ctypes route (A/B of the host overhead); so does GSR_LIBRARY naming another build of libgsr (the
module is linked against the in-tree libgsr.so, the ctypes route loads the named one)."""
import hashlib
import importlib.util
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
_ROOT = os.path.dirname(_PKG)
BUILD = os.path.join(_ROOT, "build", "ext_host")
NAME = "gsr_host"
SOURCE = os.path.join(_PKG, "csrc", "host_ext.cpp")


def so_path():
    return os.path.join(BUILD, NAME + ".so")


def source_digest():
    """Hash of the sources the module is built from (a stale build is not loaded)."""
    h = hashlib.sha256()
    for p in (SOURCE, os.path.join(_ROOT, "include", "gsr.h"), os.path.join(_ROOT, "include", "gsr_train.h")):
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build(verbose=False):
    import torch.utils.cpp_extension as ce
    os.makedirs(BUILD, exist_ok=True)
    ce.load(name=NAME, sources=[SOURCE], build_directory=BUILD, with_cuda=False, verbose=verbose,
            extra_include_paths=[os.path.join(_ROOT, "include"), "/opt/rocm/include"],
            extra_cflags=["-O2", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"],
            extra_ldflags=["-L" + _HERE, "-lgsr", "-Wl,-rpath," + _HERE, "-L/opt/rocm/lib", "-lamdhip64",
                           "-lc10_hip", "-ltorch_hip"])
    with open(os.path.join(BUILD, "source.sha"), "w") as f:
        f.write(source_digest())
    return so_path()


def load():
    if os.environ.get("GSR_HOST_EXT", "1") == "0":
        return None
    lib = os.environ.get("GSR_LIBRARY")
    if lib and os.path.realpath(lib) != os.path.realpath(os.path.join(_HERE, "libgsr.so")):
        return None  # a variant library (GSR_LIBRARY): the module links the in-tree libgsr.so
    path = so_path()
    try:
        with open(os.path.join(BUILD, "source.sha")) as f:
            built = f.read().strip()
    except OSError:
        return None  # not built: the ctypes route
    if not os.path.exists(path) or built != source_digest():
        return None  # built from other sources: the ctypes route
    spec = importlib.util.spec_from_file_location(NAME, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod
