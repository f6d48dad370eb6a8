"""CPU: the C-ABI library loads, exports every symbol include/nlh.h declares,
host-only entry points behave, and device entry points fail loudly (no CPU
fallback) when no GPU is visible."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT, gpu_available

import nonlocalheatequation_amd as N

HEADER = os.path.join(ROOT, "include", "nlh.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nlh(?:1d)?_[a-z_]+)\s*\(", text)))


def test_header_symbols_exported():
    syms = declared_symbols()
    assert len(syms) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", N.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (nlh(?:1d)?_\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_python_binding_covers_header():
    assert set(declared_symbols()) == set(N._SIGNATURES)  # noqa: SLF001
    N.lib()


def test_abi_version():
    assert N.lib().nlh_abi_version() == 6


def test_params_layout_matches_header():
    # the ctypes mirror must have the C struct's size (offsets checked by a tiny C probe)
    src = os.path.join(ROOT, "build", "probe_layout.c")
    os.makedirs(os.path.dirname(src), exist_ok=True)
    with open(src, "w") as f:
        f.write('#include <stdio.h>\n#include <stddef.h>\n#include "nlh.h"\n'
                'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(nlh_params),'
                ' offsetof(nlh_params, tiles_x), offsetof(nlh_params, comm_id),'
                ' sizeof(nlh_info), offsetof(nlh_info, arch), offsetof(nlh_info, steps_per_pass)); return 0;}\n')
    exe = os.path.join(ROOT, "build", "probe_layout")
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
    vals = list(map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()))
    assert vals == [ctypes.sizeof(N._Params), N._Params.tiles_x.offset, N._Params.comm_id.offset,  # noqa: SLF001
                    ctypes.sizeof(N._Info), N._Info.arch.offset, N._Info.steps_per_pass.offset]  # noqa: SLF001


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_no_cpu_fallback():
    with pytest.raises(N.NLHError, match="no HIP device"):
        N.Solver(50, 50, 5)


def test_bad_arguments_rejected_before_device():
    for kw in [dict(nx=0, ny=5, eps=1), dict(nx=10, ny=10, eps=0)]:
        with pytest.raises(N.NLHError):
            N.Solver(kw["nx"], kw["ny"], kw["eps"])
    with pytest.raises(N.NLHError, match="divide"):
        N.Solver(10, 10, 2, tiles=(3, 1))


def test_halo_plan_single_block_is_empty():
    assert N.halo_plan(64, 64, 8).shape == (0, 8)
    assert N.block_plan(64, 64, 8).tolist() == [[0, 0, 0, 0, 64, 64]]


def test_partition_file_format():
    # --file format (src/2d_nonlocal_distributed.cpp:476-484) of the reference fixtures
    from conftest import read_input
    for name in ["4s_2n", "25s_2n", "25s_4n", "25s_8n"]:
        tok = read_input(f"load_balance_{name}.txt").split()
        nx, ny, npx, npy = map(int, tok[:4])
        float(tok[4])
        assert len(tok) == 5 + 3 * npx * npy
        owners = [int(v) for v in tok[7::3]]
        nl = int(name.split("_")[1][:-1])
        assert max(owners) < nl
        own = N.resolve_owner(npx, npy, nl, [0] * (npx * npy))
        assert len(own) == npx * npy
