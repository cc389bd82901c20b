"""tools/gen_models.py --urdf: a robot outside the bundled arms gets compile-time tables (GRiD's per-robot
codegen) -- here a branched 4-joint tree with a prismatic joint.  The generated header must
carry the robot's tables with its topology (chain = 0), its exact-match test and a dispatch case with the
general-topology instantiation, and must compile (hipcc -fsyntax-only on a unit that includes it)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TREE = """<robot name="tree"><link name="base"/>
<joint name="j1" type="revolute"><parent link="base"/><child link="a"/><origin xyz="0 0 0" rpy="0 0 0"/><axis xyz="0 0 1"/></joint>
<link name="a"><origin xyz="0 0.5 0" rpy="0 0 0"/><inertial><mass value="0.3"/><inertia ixx="0.01" ixy="0" ixz="0" iyy="0.02" iyz="0" izz="0.03"/></inertial></link>
<joint name="j2" type="revolute"><parent link="a"/><child link="b"/><origin xyz="0 1 0" rpy="0.3 0 0"/><axis xyz="0 1 0"/></joint>
<link name="b"><origin xyz="0 0.4 0.1" rpy="0 0 0"/><inertial><mass value="0.2"/><inertia ixx="0.01" ixy="0" ixz="0" iyy="0.01" iyz="0" izz="0.02"/></inertial></link>
<joint name="j3" type="revolute"><parent link="a"/><child link="c"/><origin xyz="0.2 1 0" rpy="0 0 0.2"/><axis xyz="1 0 0"/></joint>
<link name="c"><origin xyz="0.1 0.3 0" rpy="0 0 0"/><inertial><mass value="0.25"/><inertia ixx="0.02" ixy="0" ixz="0" iyy="0.01" iyz="0" izz="0.02"/></inertial></link>
<joint name="j4" type="prismatic"><parent link="c"/><child link="d"/><origin xyz="0 0.5 0" rpy="0 0 0"/><axis xyz="0 0 1"/></joint>
<link name="d"><origin xyz="0 0.1 0" rpy="0 0 0"/><inertial><mass value="0.1"/><inertia ixx="0.01" ixy="0" ixz="0" iyy="0.01" iyz="0" izz="0.01"/></inertial></link>
</robot>"""


def test_user_urdf_gets_compiled_tables(tmp_path):
    urdf = tmp_path / "tree.urdf"
    urdf.write_text(TREE)
    out = tmp_path / "tmpc_models.h"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_models.py"), "--urdf", str(urdf),
                        "--out", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    h = out.read_text()
    assert "struct Robot8 {" in h and "static constexpr int chain = 0;" in h and "branched" in h
    assert "if (same_model<Robot8>(m)) return Robot8::ID;" in h
    assert "case Robot8::ID: LAUNCH<Robot8::n, (Robot8::chain != 0), Robot8>::CALL;" in h
    # the bundled tables are unchanged
    bundled = open(os.path.join(ROOT, "trajoptmpcreference_amd", "csrc", "tmpc_models.h")).read()
    assert h.startswith(bundled.split("// exact field-by-field")[0].rstrip())
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    unit = tmp_path / "unit.hip"
    unit.write_text('#include "tmpc_models.h"\nint probe(const tmpc::ModelDev& m) { return tmpc::match_static_model(m); }\n')
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-I", str(tmp_path), "-I",
                        os.path.join(ROOT, "trajoptmpcreference_amd", "csrc"), str(unit)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_too_many_joints_refused(tmp_path):
    from trajoptmpcreference_amd.urdf import planar_arm_urdf
    urdf = tmp_path / "arm8.urdf"
    urdf.write_text(planar_arm_urdf(8))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_models.py"), "--urdf", str(urdf),
                        "--out", str(tmp_path / "h.h")], capture_output=True, text=True)
    assert r.returncode != 0 and "n <= 7" in (r.stderr + r.stdout)
