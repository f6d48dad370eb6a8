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
    assert N.lib().nlh_abi_version() == 10


def test_build_id_matches_sources():
    # the library under test was built from this tree's sources and flags
    assert N.build_id() == N.source_build_id()


def test_no_diagnostic_kernels_in_library():
    """libnlh ships only result-producing kernels: no ablation instance
    (ABL != 0) of k_pair_split / k_fast / k_wide and none of the alternate
    two-step designs (tools/pair_variants.h, harness only)."""
    blob = open(N.lib_path(), "rb").read()
    names = set(re.findall(rb"_ZN3nlh\d+k_\w+", blob))
    assert any(b"k_pair_split" in n for n in names)
    for n in names:
        s = n.decode()
        assert "k_pair_mw" not in s and "k_pair_pf" not in s and "6k_pairI" not in s, s
        m = re.search(r"12k_pair_splitILi\d+ELi\d+ELi(\d+)E", s)
        assert not m or m.group(1) == "0", s
        m = re.search(r"6k_fastILi\d+ELi\d+ELi\d+ELb[01]ELi(\d+)E", s)
        assert not m or m.group(1) == "0", s


@pytest.mark.parametrize("var,val,msg", [("NLH_ABLATE", "1", "ablation"), ("NLH_PAIR_ABLATE", "12408", "ablation"),
                                         ("NLH_PAIR_SPLIT", "2", "NLH_PAIR_SPLIT"),
                                         ("NLH_SCHED", "7", "NLH_SCHED"), ("NLH_FAST_R", "x", "NLH_FAST_R")])
def test_env_rejected_before_device(monkeypatch, var, val, msg):
    # nlh_create validates the environment before it looks for a device, so
    # no setting can make the product library compute something else
    monkeypatch.setenv(var, val)
    with pytest.raises(N.NLHError, match=msg):
        N.Solver(50, 50, 5)


def test_params_layout_matches_header():
    # the ctypes mirror must have the C struct's size (offsets checked by a tiny C probe)
    src = os.path.join(ROOT, "build", "probe_layout.c")
    os.makedirs(os.path.dirname(src), exist_ok=True)
    with open(src, "w") as f:
        f.write('#include <stdio.h>\n#include <stddef.h>\n#include "nlh.h"\n'
                'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(nlh_params),'
                ' offsetof(nlh_params, tiles_x), offsetof(nlh_params, comm_id),'
                ' sizeof(nlh_info), offsetof(nlh_info, arch), offsetof(nlh_info, steps_per_pass));'
                ' printf("%zu %zu %zu %zu\\n", offsetof(nlh_info, comm_nranks), offsetof(nlh_info, comm_rank),'
                ' sizeof(nlh_phase_times), offsetof(nlh_phase_times, passes));'
                ' printf("%zu %zu\\n", sizeof(nlh_host_times), offsetof(nlh_host_times, sync_mode)); return 0;}\n')
    exe = os.path.join(ROOT, "build", "probe_layout")
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
    vals = list(map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()))
    assert vals == [ctypes.sizeof(N._Params), N._Params.tiles_x.offset, N._Params.comm_id.offset,  # noqa: SLF001
                    ctypes.sizeof(N._Info), N._Info.arch.offset, N._Info.steps_per_pass.offset,  # noqa: SLF001
                    N._Info.comm_nranks.offset, N._Info.comm_rank.offset,  # noqa: SLF001
                    ctypes.sizeof(N._PhaseTimes), N._PhaseTimes.passes.offset,  # noqa: SLF001
                    ctypes.sizeof(N._HostTimes), N._HostTimes.sync_mode.offset]  # noqa: SLF001


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
