"""Packaging for xdot (and the ``distributed_dot_product`` import shim).

``pip install . --no-build-isolation`` (or ``python setup.py bdist_wheel``) compiles the gfx950
HIP extension with ``xdot/build.py`` (``hipcc --offload-arch=gfx950``, no hipify, no JIT) and
ships ``xdot/_C.so`` inside the package; the version comes from ``xdot.VERSION_INFO``, read
without importing the package (reference: ``setup.py:17-64``, which reads it the same way).
``XDOT_SKIP_NATIVE=1`` packages the pure-Python parts only (CPU use; GPU ops then raise).
"""
import ast
import importlib.util
import os

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution

HERE = os.path.abspath(os.path.dirname(__file__))


def get_version(module="xdot"):
    with open(os.path.join(HERE, module, "__init__.py")) as f:
        for line in f:
            if line.startswith("VERSION_INFO"):
                return ".".join(map(str, ast.literal_eval(line.split("=")[-1].strip())))
    raise RuntimeError("VERSION_INFO not found")


class BuildWithHip(build_py):
    """Compile xdot/_C.so for gfx950 before the Python files are collected."""

    def run(self):
        if os.environ.get("XDOT_SKIP_NATIVE", "0") != "1":
            spec = importlib.util.spec_from_file_location("_xdot_build", os.path.join(HERE, "xdot", "build.py"))
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            path = mod.build(verbose=False, jobs=int(os.environ.get("MAX_JOBS", "4")))
            print(f"xdot: built {path}")
        super().run()


class BinaryDistribution(Distribution):
    def has_ext_modules(self):  # platform wheel: ships a gfx950 code object
        return os.environ.get("XDOT_SKIP_NATIVE", "0") != "1"


with open(os.path.join(HERE, "README.md")) as f:
    long_description = f.read()

setup(
    name="xdot",
    version=get_version(),
    description="Sequence-parallel distributed dot-product attention for AMD Instinct MI355X "
                "(gfx950 HIP kernels, RCCL over xGMI)",
    long_description=long_description,
    long_description_content_type="text/markdown",
    keywords=["transformer", "attention", "sequence-parallel", "rocm", "mi355x"],
    license="MIT",
    packages=find_packages(include=["xdot", "xdot.*", "distributed_dot_product", "distributed_dot_product.*"]),
    package_data={"xdot": ["_C.so"]},
    python_requires=">=3.9",
    install_requires=["torch"],
    cmdclass={"build_py": BuildWithHip},
    distclass=BinaryDistribution,
    classifiers=[
        "Programming Language :: Python :: 3",
        "Operating System :: POSIX :: Linux",
        "Environment :: GPU",
    ],
)
