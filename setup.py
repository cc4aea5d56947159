"""Build hook for ``pip install --no-build-isolation [-e] .``: compiles every HIP kernel for gfx950
(``replicann_amd/_build.py``: hipcc --offload-arch=gfx950, hash-keyed incremental objects) into
``replicann_amd/_C.so`` plus the host runtime ``_io.so`` BEFORE the package files are collected,
so both the wheel and an editable (develop) install carry the extension.  Metadata lives in
pyproject.toml; it is read here too because setuptools < 61 ignores its [project] table."""

import importlib.util
import os

from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.command.develop import develop

ROOT = os.path.dirname(os.path.abspath(__file__))


def _native_build():
    if os.environ.get("REPLICANN_SKIP_NATIVE") == "1":  # metadata-only builds
        return
    # load the builder by path: importing the package would import torch-dependent modules first
    spec = importlib.util.spec_from_file_location("_rn_build", os.path.join(ROOT, "replicann_amd", "_build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.build(verbose=True)


class BuildPy(build_py):
    def run(self):
        _native_build()
        super().run()


class Develop(develop):
    def run(self):
        _native_build()
        super().run()


def _meta():
    try:
        import tomli
    except ImportError:  # pragma: no cover
        return {}
    with open(os.path.join(ROOT, "pyproject.toml"), "rb") as f:
        pp = tomli.load(f)
    p, t = pp["project"], pp.get("tool", {}).get("setuptools", {})
    return dict(name=p["name"], version=p["version"], description=p["description"],
                python_requires=p["requires-python"], install_requires=p["dependencies"],
                extras_require=p.get("optional-dependencies", {}), packages=t.get("packages"),
                package_data=t.get("package-data"), include_package_data=True,
                entry_points={"console_scripts": [f"{k} = {v}" for k, v in p.get("scripts", {}).items()]})


setup(cmdclass={"build_py": BuildPy, "develop": Develop}, **_meta())
