"""The C++ plugin (include/ompl_amd/NearestNeighborsGPU.h) compiles against the OMPL
interface — the standalone surface and, where the reference tree is present, the
reference's own datastructures/NearestNeighbors.h — and on the GPU answers planner-style
queries identically to the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "plugin_test.cpp")
MV_SRC = os.path.join(ROOT, "tests", "cpp", "mv_plugin_test.cpp")
BOUNDARY_SRC = os.path.join(ROOT, "tests", "cpp", "boundary_test.cpp")
REF_SRC = "/root/reference/src"


def _build(out, extra, src=SRC):
    cmd = ["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"), *extra, src, "-o", out,
           "-L", os.path.join(ROOT, "ompl_amd", "lib"), "-L", os.path.join(ROOT, "oracle"), "-lompl_gpu", "-loracle",
           f"-Wl,-rpath,{os.path.join(ROOT, 'ompl_amd', 'lib')}", f"-Wl,-rpath,{os.path.join(ROOT, 'oracle')}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def test_plugin_compiles_standalone(tmp_path):
    exe = _build(str(tmp_path / "plugin_sa"), [])
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0 and "PLUGIN COMPILED" in r.stdout


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SRC, "ompl/datastructures/NearestNeighbors.h")),
                    reason="reference sources absent")
def test_plugin_compiles_against_reference_interface(tmp_path):
    _build(str(tmp_path / "plugin_ref"), ["-DOMPL_AMD_WITH_OMPL", "-I", REF_SRC])


@pytest.mark.gpu
def test_plugin_runs_on_gpu(tmp_path, gpu):
    exe = _build(str(tmp_path / "plugin_run"), [])
    r = subprocess.run([exe, "run"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "PLUGIN OK" in r.stdout, r.stdout + r.stderr


def test_motion_validator_plugin_compiles_standalone(tmp_path):
    exe = _build(str(tmp_path / "mv_sa"), [], MV_SRC)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0 and "MV PLUGIN COMPILED" in r.stdout


@pytest.mark.gpu
def test_motion_validator_plugin_runs_on_gpu(tmp_path, gpu):
    exe = _build(str(tmp_path / "mv_run"), [], MV_SRC)
    r = subprocess.run([exe, "run"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "MV PLUGIN OK" in r.stdout, r.stdout + r.stderr


def test_boundary_compiles_and_rng_streams(tmp_path):
    """Standalone ompl::RNG: the seed stream after RNG::setSeed(42) and the uniformReal stream
    equal the oracle's restatement (CPU only)."""
    exe = _build(str(tmp_path / "boundary_sa"), [], BOUNDARY_SRC)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0 and "BOUNDARY COMPILED" in r.stdout, r.stdout + r.stderr
    r = subprocess.run([exe, "rng"], capture_output=True, text=True)
    assert r.returncode == 0 and "BOUNDARY RNG OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_boundary_runs_on_gpu(tmp_path, gpu):
    """One RNG seed per NearestNeighborsGPU, setDistanceFunction verification, the
    StateValidityChecker plugin (host == device == oracle) and the SelfConfig hook."""
    exe = _build(str(tmp_path / "boundary_run"), [], BOUNDARY_SRC)
    r = subprocess.run([exe, "run"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "BOUNDARY OK" in r.stdout, r.stdout + r.stderr


VERTEX_SRC = os.path.join(ROOT, "tests", "cpp", "vertex_plugin_test.cpp")


def test_vertex_plugin_compiles_standalone(tmp_path):
    """NearestNeighborsGPU<std::size_t> + ElementPacker (PRM Vertex / Blaze VertexID) compiles."""
    exe = _build(str(tmp_path / "vertex_sa"), [], VERTEX_SRC)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0 and "VERTEX PLUGIN COMPILED" in r.stdout


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SRC, "ompl/datastructures/NearestNeighbors.h")),
                    reason="reference sources absent")
def test_vertex_plugin_compiles_against_reference_interface(tmp_path):
    _build(str(tmp_path / "vertex_ref"), ["-DOMPL_AMD_WITH_OMPL", "-I", REF_SRC], VERTEX_SRC)


@pytest.mark.gpu
def test_vertex_plugin_runs_on_gpu(tmp_path, gpu):
    """PRM*-style causal nearestK over vertex ids, Blaze-style nearestR, removal, batched kNN."""
    exe = _build(str(tmp_path / "vertex_run"), [], VERTEX_SRC)
    r = subprocess.run([exe, "run"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "VERTEX PLUGIN OK" in r.stdout, r.stdout + r.stderr
