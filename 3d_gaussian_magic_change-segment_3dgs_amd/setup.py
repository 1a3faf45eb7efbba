"""pip-installable gsr: the reference's build glue (DGR/setup.py:17-34, installed by
environment.yml:16) for the MI355X rasterizer.

    pip install --no-build-isolation ./3d_gaussian_magic_change-segment_3dgs_amd

installs `diff_gaussian_rasterization` (the drop-in API; `gaussian_renderer/__init__.py`
imports it unchanged), `gsr_train` and `gsr_tools`, with libgsr.so (hand-written HIP for
gfx950, built by csrc/Makefile with hipcc) inside the `diff_gaussian_rasterization`
package, where `_C.py` loads it from.  `--no-build-isolation` as for the reference's
CUDAExtension: the build runs against the installed torch, and there is no package index
to fetch an isolated build environment from.

GSR_ARCH overrides the offload target (default gfx950).
"""
import os
import shutil
import subprocess

from setuptools import setup
from setuptools.command.build_py import build_py

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = "libgsr.so"


class BuildWithLibgsr(build_py):
    """Runs csrc/Makefile (incremental: the in-tree libgsr.so is rebuilt only when a source
    changed) and ships the library inside the diff_gaussian_rasterization package."""

    def run(self):
        jobs = str(min(16, os.cpu_count() or 1))
        cmd = ["make", "-j", jobs, "-C", os.path.join(HERE, "csrc")]
        if os.environ.get("GSR_ARCH"):
            cmd.append("ARCH=" + os.environ["GSR_ARCH"])
        subprocess.check_call(cmd)
        super().run()
        dst = os.path.join(self.build_lib, "diff_gaussian_rasterization")
        os.makedirs(dst, exist_ok=True)
        shutil.copy2(os.path.join(HERE, "diff_gaussian_rasterization", LIB), os.path.join(dst, LIB))


setup(
    name="diff_gaussian_rasterization",
    version="0.1.0+gsr.gfx950",
    description="MI355X (gfx950) differentiable Gaussian rasterizer behind the "
                "diff_gaussian_rasterization API",
    packages=["diff_gaussian_rasterization", "gsr_train", "gsr_tools"],
    package_dir={"": "."},
    package_data={"diff_gaussian_rasterization": [LIB]},
    cmdclass={"build_py": BuildWithLibgsr},
    python_requires=">=3.8",
    zip_safe=False,
)
