"""CPU-side check of the drop-in boundary: include/lcfir/FilterCore.h gives a
NON-template Diskerror::apply_filter_range with the reference's parameter
types (FilterCore.h:20-27), so ProcessFile.cp:71-78's call shape -- the
function passed by name to std::thread -- compiles against it.  The GPU run of
the same program is tests/test_gpu_cpp_dropin.py::test_reference_call_shape."""
import os
import subprocess

from conftest import ROOT

INC = os.path.join(ROOT, "include")
SRC = os.path.join(ROOT, "tests", "cpp", "dropin_processfile.cpp")


import pytest


@pytest.mark.parametrize("std", ["c++17", "c++20", "c++2b"])
def test_reference_call_shape_compiles(std):
    """The reference builds as C++23 (Makefile STD; c++2b is g++ 11's name
    for it); the drop-in headers compile clean in that mode and the older ones."""
    r = subprocess.run(["g++", "-std=" + std, "-fsyntax-only", "-Wall", "-Wextra", "-I", INC, SRC],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


def test_template_form_alone_is_not_enough(tmp_path):
    """The failure the VERDICT reproduced: a function TEMPLATE passed by name to
    std::thread does not compile -- hence the non-template header."""
    src = tmp_path / "t.cpp"
    src.write_text(
        '#include <thread>\n#include <vector>\n#include "lcfir/FilterCore.hpp"\n'
        'struct P { void report(size_t) {} };\n'
        'int main() { std::vector<float> a(8), b(8); std::vector<double> h(3); P p;\n'
        '  std::thread t(lcfir::apply_filter_range, std::cref(a), std::cref(h), std::ref(b),\n'
        '                (int_fast64_t)0, (int_fast64_t)8, &p); t.join(); }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", INC, str(src)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
