"""URDF -> rigid-body model arrays (host side, one-time).

Restates the conventions of the reference's GRiD URDF parser so that the
arrays handed to the device are the ones the reference's RBD code sees:

* links/joints in document order (`URDFParser.parse_links/parse_joints`,
  GRiD/URDFParser/URDFParser.py:258-320);
* fixed joints are folded into their parent (`remove_fixed_joints`, :323-345):
  grandchild transforms are right-multiplied by the fixed joint's transform
  and the child inertia is added as X^T I X;
* depth-first renumbering from the root (`dfs_order_update`, :366-381), so the
  joint/link id of a body is its DFS position and parent ids precede children;
* the joint transform is X(q) = Xfree(q) * Xfixed with Xfixed = rot(E) xlt(r),
  E = rx(roll) ry(pitch) rz(yaw) (SpatialAlgebra.py:66-70,89-103,
  Joint.py:52-97), and every float coefficient of the product is snapped with
  `nsimplify(tolerance=1e-6, rational=True)` (Joint.py:90), i.e.
  `Rational(f).limit_denominator(10**6)`;
* spatial inertia built from the *link-level* <origin> translation (not the
  <inertial> origin), with the same 1e-12 snapping of the COM skew matrix and
  zeroing of |entries| <= 1e-10 (Link.py:48-63).

Instead of a SymPy expression per joint we keep X as an affine combination of
constant 6x6 coefficient matrices, exactly what the snapped expression is:

    revolute:   X(q) = X0 + cos(q) * Xa + sin(q) * Xb
    prismatic:  X(q) = X0 + q * Xa

so evaluating X on the device needs one sincos per joint and no symbolic code
(the reference lambdifies on every call: SURVEY F11).
"""
from dataclasses import dataclass, field
from fractions import Fraction
import math
import xml.etree.ElementTree as ET

import numpy as np

JTYPE_REVOLUTE = 0
JTYPE_PRISMATIC = 1


def _snap(v: float, max_den: int) -> float:
    """`nsimplify(Float, tolerance=1/max_den, rational=True)` then evalf."""
    if v == 0.0:
        return 0.0
    return float(Fraction(v).limit_denominator(max_den))


def _skew(x, y, z):
    return np.array([[0.0, -z, y], [z, 0.0, -x], [-y, x, 0.0]])


def _rx(t):
    c, s = math.cos(t), math.sin(t)
    return np.array([[1.0, 0.0, 0.0], [0.0, c, s], [0.0, -s, c]])


def _ry(t):
    c, s = math.cos(t), math.sin(t)
    return np.array([[c, 0.0, -s], [0.0, 1.0, 0.0], [s, 0.0, c]])


def _rz(t):
    c, s = math.cos(t), math.sin(t)
    return np.array([[c, s, 0.0], [-s, c, 0.0], [0.0, 0.0, 1.0]])


def _rot(E):
    X = np.zeros((6, 6))
    X[:3, :3] = E
    X[3:, 3:] = E
    return X


def _xlt(r3):
    X = np.eye(6)
    X[3:, :3] = -r3
    return X


# The rotation-about-axis matrices as cos/sin/const coefficient triples.
def _axis_coeffs(axis_idx):
    """rot(r_axis(theta)) = C0 + cos*Ca + sin*Cb (SpatialAlgebra.py:78-97)."""
    C0, Ca, Cb = np.zeros((3, 3)), np.zeros((3, 3)), np.zeros((3, 3))
    if axis_idx == 2:      # rz: [[c, s, 0], [-s, c, 0], [0, 0, 1]]
        Ca[0, 0] = Ca[1, 1] = 1.0
        Cb[0, 1], Cb[1, 0] = 1.0, -1.0
        C0[2, 2] = 1.0
    elif axis_idx == 1:    # ry: [[c, 0, -s], [0, 1, 0], [s, 0, c]]
        Ca[0, 0] = Ca[2, 2] = 1.0
        Cb[0, 2], Cb[2, 0] = -1.0, 1.0
        C0[1, 1] = 1.0
    else:                  # rx: [[1, 0, 0], [0, c, s], [0, -s, c]]
        Ca[1, 1] = Ca[2, 2] = 1.0
        Cb[1, 2], Cb[2, 1] = 1.0, -1.0
        C0[0, 0] = 1.0
    return _rot(C0), _rot(Ca), _rot(Cb)


@dataclass
class _Joint:
    name: str
    parent: str
    child: str
    jtype: str
    axis: tuple
    xyz: tuple
    rpy: tuple
    damping: float = 0.0
    # X(q) = X0 + a(q)*Xa + b(q)*Xb   (a,b) = (cos,sin) or (q,0)
    X0: np.ndarray = None
    Xa: np.ndarray = None
    Xb: np.ndarray = None
    S: np.ndarray = None
    # homogeneous 4x4 transform H(q) = H0 + a(q)*Ha + b(q)*Hb (Joint.py:91-95)
    H0: np.ndarray = None
    Ha: np.ndarray = None
    Hb: np.ndarray = None


@dataclass
class RobotModel:
    """Model arrays in DFS order (index = joint id = child-link id)."""
    name: str
    n: int
    parent: np.ndarray                     # (n,) int32, -1 = base
    jtype: np.ndarray                      # (n,) int32, JTYPE_*
    S: np.ndarray                          # (n, 6) motion subspace (unit vector)
    X0: np.ndarray                         # (n, 6, 6)
    Xa: np.ndarray                         # (n, 6, 6)
    Xb: np.ndarray                         # (n, 6, 6)
    I: np.ndarray                          # (n, 6, 6) spatial inertia
    damping: np.ndarray                    # (n,)
    subtree: list = field(default_factory=list)   # sorted subtree ids (Robot.py:67-68)
    joint_names: list = field(default_factory=list)
    H0: np.ndarray = None                  # (n, 4, 4) homogeneous transform coefficients
    Ha: np.ndarray = None                  #   H(q) = H0 + cos q Ha + sin q Hb (revolute)
    Hb: np.ndarray = None                  #   H(q) = H0 + q Ha (prismatic)

    @property
    def nq(self):
        return self.n

    def X(self, j: int, q: float) -> np.ndarray:
        if self.jtype[j] == JTYPE_REVOLUTE:
            return self.X0[j] + math.cos(q) * self.Xa[j] + math.sin(q) * self.Xb[j]
        return self.X0[j] + q * self.Xa[j]

    def H(self, j: int, q: float) -> np.ndarray:
        """Robot.get_Xmat_hom_Func_by_id (Joint.py:105-106)."""
        if self.jtype[j] == JTYPE_REVOLUTE:
            return self.H0[j] + math.cos(q) * self.Ha[j] + math.sin(q) * self.Hb[j]
        return self.H0[j] + q * self.Ha[j]

    def dH(self, j: int, q: float) -> np.ndarray:
        """Robot.get_dXmat_hom_Func_by_id: d/dq of H (Joint.py:97,111-112)."""
        if self.jtype[j] == JTYPE_REVOLUTE:
            return -math.sin(q) * self.Ha[j] + math.cos(q) * self.Hb[j]
        return self.Ha[j].copy()

    def is_serial_chain(self) -> bool:
        return all(int(self.parent[j]) == j - 1 for j in range(self.n))


def _floats(s, default="0 0 0"):
    return [float(v) for v in (s if s is not None else default).split()]


def _spatial_inertia(mass, inertia6, xyz):
    """Link.build_spatial_inertia (Link.py:48-63)."""
    r = np.array([[_snap(v, 10 ** 12) for v in row] for row in _skew(*xyz)])
    ixx, ixy, ixz, iyy, iyz, izz = inertia6
    I3 = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]])
    mc = mass * r
    mccT = mc @ r.T
    top = np.hstack((I3 + mccT, mc))
    bot = np.hstack((mc.T, mass * np.eye(3)))
    Im = np.vstack((top, bot)).astype(float)
    Im[np.isclose(Im, np.zeros((6, 6)), 1e-10, 1e-10)] = 0.0
    return Im


def _joint_transform(j: _Joint):
    """Xfree(q) * Xfixed as coefficient matrices, snapped like Joint.py:88-90."""
    E = _rx(j.rpy[0]) @ _ry(j.rpy[1]) @ _rz(j.rpy[2])
    Xfixed = _rot(E) @ _xlt(_skew(*j.xyz))
    if j.jtype == "revolute":
        ax = _axis_index(j.axis)
        C0, Ca, Cb = _axis_coeffs(ax)
        S = np.zeros(6)
        S[ax] = 1.0
        X0, Xa, Xb = C0 @ Xfixed, Ca @ Xfixed, Cb @ Xfixed
    elif j.jtype == "prismatic":
        ax = _axis_index(j.axis)
        # xlt(skew(theta*e_ax)) = I + theta * D  (Joint.py:68-80)
        e = [0.0, 0.0, 0.0]
        e[ax] = 1.0
        D = _xlt(_skew(*e)) - np.eye(6)
        S = np.zeros(6)
        S[3 + ax] = 1.0
        X0, Xa, Xb = Xfixed.copy(), D @ Xfixed, np.zeros((6, 6))
    elif j.jtype == "fixed":
        S = np.zeros(6)
        X0, Xa, Xb = Xfixed.copy(), np.zeros((6, 6)), np.zeros((6, 6))
    else:
        raise ValueError(f"joint '{j.name}': only revolute, prismatic and fixed joints are supported "
                         f"(GRiD/URDFParser/Joint.py:85-87)")
    snap = np.vectorize(lambda v: _snap(float(v), 10 ** 6))
    return snap(X0), snap(Xa), snap(Xb), S


def _hom(R3, t3):
    H = np.zeros((4, 4))
    H[:3, :3] = R3
    H[:3, 3] = t3
    return H


def _joint_hom(j: _Joint):
    """Homogeneous transform coefficients (Joint.py:91-95): rotation (Rfree(q) E)^T,
    translation = free translation + origin xyz, snapped like nsimplify(tolerance=1e-6)."""
    E = _rx(j.rpy[0]) @ _ry(j.rpy[1]) @ _rz(j.rpy[2])
    xyz = np.array(j.xyz, dtype=float)
    zero = np.zeros(3)
    if j.jtype == "revolute":
        C0, Ca, Cb = (C[:3, :3] for C in _axis_coeffs(_axis_index(j.axis)))
        H0, Ha, Hb = _hom((C0 @ E).T, xyz), _hom((Ca @ E).T, zero), _hom((Cb @ E).T, zero)
        H0[3, 3] = 1.0
    elif j.jtype == "prismatic":
        e = np.zeros(3)
        e[_axis_index(j.axis)] = 1.0
        H0, Ha, Hb = _hom(E.T, xyz), _hom(np.zeros((3, 3)), e), np.zeros((4, 4))
        H0[3, 3] = 1.0
    else:
        H0, Ha, Hb = _hom(E.T, xyz), np.zeros((4, 4)), np.zeros((4, 4))
        H0[3, 3] = 1.0
    snap = np.vectorize(lambda v: _snap(float(v), 10 ** 6))
    return snap(H0), snap(Ha), snap(Hb)


def _axis_index(axis):
    # the reference tests axis[2]==1, then axis[1]==1, then axis[0]==1 (Joint.py:56-80)
    for idx in (2, 1, 0):
        if axis[idx] == 1:
            return idx
    raise ValueError(f"joint axis {axis}: only +x/+y/+z unit axes are supported (Joint.py:56-80)")


def parse_urdf(path_or_text: str) -> RobotModel:
    """Parse a URDF file (or an XML string) into DFS-ordered model arrays."""
    text = path_or_text
    if not path_or_text.lstrip().startswith("<"):
        with open(path_or_text, "r", errors="ignore") as f:
            text = f.read()
    root = ET.fromstring(text)

    links = []          # (name, mass, inertia6, xyz)
    for raw in root.findall(".//link"):
        o = raw.find("origin")
        xyz = _floats(o.get("xyz", "0 0 0")) if o is not None else [0.0, 0.0, 0.0]
        inert = raw.find("inertial")
        if inert is None:
            mass, i6 = 0.0, (0.0,) * 6
        else:
            ri = inert.find("inertia")
            mass = float(inert.find("mass").get("value", "0"))
            i6 = tuple(float(ri.get(k, "0")) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz"))
        links.append([raw.get("name"), _spatial_inertia(mass, i6, xyz)])
    link_I = {name: I for name, I in links}

    joints = []
    for raw in root.findall(".//joint"):
        o = raw.find("origin")
        ax = raw.find("axis")
        dyn = raw.find("dynamics")
        j = _Joint(name=raw.get("name"), parent=raw.find("parent").get("link"),
                   child=raw.find("child").get("link"), jtype=raw.get("type"),
                   axis=tuple(_floats(ax.get("xyz"))) if ax is not None else (0.0, 0.0, 0.0),
                   xyz=tuple(_floats(o.get("xyz") if o is not None else None)),
                   rpy=tuple(_floats(o.get("rpy") if o is not None else None)),
                   damping=float(dyn.get("damping")) if dyn is not None else 0.0)
        j.X0, j.Xa, j.Xb, j.S = _joint_transform(j)
        if j.jtype in ("revolute", "prismatic", "fixed"):
            j.H0, j.Ha, j.Hb = _joint_hom(j)
        joints.append(j)

    # fold fixed joints (URDFParser.py:323-345)
    for j in list(joints):
        if j.jtype != "fixed":
            continue
        for gc in joints:
            if gc.parent == j.child:
                gc.parent = j.parent
                gc.X0, gc.Xa, gc.Xb = gc.X0 @ j.X0, gc.Xa @ j.X0, gc.Xb @ j.X0
                gc.H0, gc.Ha, gc.Hb = j.H0 @ gc.H0, j.H0 @ gc.Ha, j.H0 @ gc.Hb
        Xf = j.X0
        link_I[j.parent] = link_I[j.parent] + Xf.T @ link_I[j.child] @ Xf
        joints.remove(j)
        link_I.pop(j.child)

    children = {j.child for j in joints}
    roots = [name for name, _ in links if name in link_I and name not in children]
    if len(roots) != 1:
        raise ValueError(f"URDF must have exactly one root link, found {roots}")
    by_name = {j.name: j for j in joints}

    order = []
    def dfs(parent_link):
        for j in joints:                       # document order (Robot.py:142-146)
            if j.parent == parent_link:
                order.append(j.name)
                dfs(j.child)
    dfs(roots[0])
    if len(order) != len(joints):
        raise ValueError("URDF joint graph is not a tree rooted at the base link "
                         f"(reached {len(order)} of {len(joints)} joints)")
    idx = {name: i for i, name in enumerate(order)}
    child_to_id = {by_name[name].child: i for name, i in idx.items()}
    n = len(order)
    parent = np.array([child_to_id.get(by_name[name].parent, -1) for name in order], dtype=np.int32)
    jt = np.array([JTYPE_REVOLUTE if by_name[nm].jtype == "revolute" else JTYPE_PRISMATIC for nm in order],
                  dtype=np.int32)
    subtree = [[i] for i in range(n)]
    for i in reversed(range(n)):
        if parent[i] >= 0:
            subtree[parent[i]] = sorted(set(subtree[parent[i]]) | set(subtree[i]))
    return RobotModel(
        name=root.get("name") or "robot", n=n, parent=parent, jtype=jt,
        S=np.array([by_name[nm].S for nm in order]),
        X0=np.array([by_name[nm].X0 for nm in order]),
        Xa=np.array([by_name[nm].Xa for nm in order]),
        Xb=np.array([by_name[nm].Xb for nm in order]),
        I=np.array([link_I[by_name[nm].child] for nm in order]),
        damping=np.array([by_name[nm].damping for nm in order]),
        subtree=[sorted(s) for s in subtree], joint_names=list(order),
        H0=np.array([by_name[nm].H0 for nm in order]),
        Ha=np.array([by_name[nm].Ha for nm in order]),
        Hb=np.array([by_name[nm].Hb for nm in order]))


def planar_arm_urdf(n_links: int, mass: float = 0.1, length: float = 1.0) -> str:
    """Serial chain of `n_links` revolute-z joints with 1 m links and 0.1 kg
    rods -- the family of models/arm{2..6}.urdf in the reference, with arm6's
    joint6 parent/child corrected.  Generated, not copied."""
    ixx = mass * (3 * (0.05 ** 2) + length ** 2) / 12.0 + 0.0  # thin-rod inertia about the COM
    izz = 0.5 * mass * (0.05 ** 2)
    parts = ['<?xml version="1.0" ?>', f'<robot name="{n_links}_link">', '  <link name="base_link"/>']
    for i in range(1, n_links + 1):
        parent = "base_link" if i == 1 else f"link{i - 1}"
        y = 0.0 if i == 1 else length
        parts += [f'  <joint name="joint{i}" type="revolute">',
                  f'    <parent link="{parent}"/>', f'    <child link="link{i}"/>',
                  f'    <origin rpy="0 0 0" xyz="0 {y:g} 0"/>', '    <axis xyz="0 0 1"/>', '  </joint>',
                  f'  <link name="link{i}">',
                  f'    <origin rpy="1.5707963267948966 0 0" xyz="0 {length / 2:g} 0"/>',
                  '    <inertial>',
                  f'      <origin rpy="1.5707963267948966 0 0" xyz="0 {length / 2:g} 0"/>',
                  f'      <mass value="{mass!r}"/>',
                  f'      <inertia ixx="{ixx!r}" ixy="0.0" ixz="0.0" iyy="{ixx!r}" iyz="0.0" izz="{izz!r}"/>',
                  '    </inertial>', '  </link>']
    parts.append('</robot>')
    return "\n".join(parts) + "\n"


def pendulum_urdf(mass: float = 1.0, length: float = 1.0, bob_inertia: float = 1e-3) -> str:
    """A pendulum: one revolute joint about x and a bob of `mass` hanging `length` below it along -z,
    so gravity (options['gravity'], along z) gives the torque -mass g length sin(q) and q = pi is
    upright.  The reference's examples/pendulum.py uses a PendulumPlant that TrajoptPlant.py never
    defines; this URDF is the model behind plant.PendulumPlant.  Generated, not copied."""
    i = bob_inertia
    return "\n".join([
        '<?xml version="1.0" ?>', '<robot name="pendulum">', '  <link name="base_link"/>',
        '  <joint name="joint1" type="revolute">', '    <parent link="base_link"/>', '    <child link="bob"/>',
        '    <origin rpy="0 0 0" xyz="0 0 0"/>', '    <axis xyz="1 0 0"/>', '  </joint>',
        # the parser takes the COM offset from the link's own <origin>, as the reference's
        # URDFParser does (Link.py:48-63); the inertial block repeats it (models/arm*.urdf style)
        '  <link name="bob">', f'    <origin rpy="0 0 0" xyz="0 0 {-length!r}"/>', '    <inertial>',
        f'      <origin rpy="0 0 0" xyz="0 0 {-length!r}"/>',
        f'      <mass value="{mass!r}"/>',
        f'      <inertia ixx="{i!r}" ixy="0.0" ixz="0.0" iyy="{i!r}" iyz="0.0" izz="{i!r}"/>',
        '    </inertial>', '  </link>', '</robot>']) + "\n"

