"""Builds the native libraries (make: gfx950 HIP + host OpenMP/BP4) before packaging."""
import subprocess

from setuptools import setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        subprocess.run(["make", "-j8", "all"], check=True)
        super().run()


setup(cmdclass={"build_py": BuildNative})
