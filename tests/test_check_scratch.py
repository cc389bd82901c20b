"""tools/check_scratch.py (make check-scratch): the parser of hipcc's kernel-resource-usage remarks
flags scratch in a hot fp64 or fp32 kernel of a compiled model and ignores the runtime-model
instances (ModelRef: any robot outside the bundled arms)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _remarks(name, vgpr, scratch):
    return (f"x.hip:1:1: remark: Function Name: {name} [-Rpass-analysis=kernel-resource-usage]\n"
            f"x.hip:1:1: remark:     VGPRs: {vgpr} [-Rpass-analysis=kernel-resource-usage]\n"
            f"x.hip:1:1: remark:     ScratchSize [bytes/lane]: {scratch} [-Rpass-analysis=kernel-resource-usage]\n"
            f"x.hip:1:1: remark:     Occupancy [waves/SIMD]: 2 [-Rpass-analysis=kernel-resource-usage]\n")


def _run(text):
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_scratch.py")], input=text,
                          capture_output=True, text=True)


def test_scratch_in_hot_fp64_kernel_fails():
    grad64 = "_ZN4tmpc9k_qp_gradILi6ELb1ENS_4Arm6EdEEvT1_NS_5PListEiidPKdPKiS5_S5_PdS8_"
    assert _run(_remarks(grad64, 168, 592)).returncode == 1
    assert _run(_remarks(grad64, 232, 0)).returncode == 0
    bwd64 = "_ZN4tmpc15k_ilqr_backwardILi6EdLb1EEEvPKNS_7CostDevE"
    assert _run(_remarks(bwd64, 108, 160)).returncode == 1


def test_scratch_in_hot_fp32_kernel_fails():
    """The fp32 instances (BASELINE configs 3 / 5) are gated too: before the full-unroll build they kept
    192-256 B per lane of scratch."""
    fwd32 = "_ZN4tmpc14k_ilqr_forwardILi6ELb1ELb1ENS_4Arm6EfLb1EEEvT2_PKNS_7CostDevE"
    assert _run(_remarks(fwd32, 231, 256)).returncode == 1
    assert _run(_remarks(fwd32, 165, 0)).returncode == 0
    minv32 = "_ZN4tmpc9k_qp_minvILi6ELb1ENS_4Arm6EfEEvT1_NS_5PListEiiPKdPKiPd"
    assert _run(_remarks(minv32, 140, 192)).returncode == 1


def test_runtime_model_instances_are_not_gated():
    ref64 = "_ZN4tmpc7k_qp_fdILi6ELb0ENS_8ModelRefEdEEvT1_NS_5PListEiidPKdS5_S5_PKiPdS8_"
    assert _run(_remarks(ref64, 256, 2176)).returncode == 0


def test_model_independent_hot_kernels_are_gated():
    ginv6 = "_ZN4tmpc11k_ginv_softILi6EEEvPKNS_7CostDevEPKNS_9ConstrDevENS_5PListEiiPKdPKiS9_S9_S9_S9_PdSB_"
    assert _run(_remarks(ginv6, 256, 1168)).returncode == 1
    assert _run(_remarks(ginv6, 120, 0)).returncode == 0
    pcg = "_ZN4tmpc10k_hard_pcgILi12ELi2EEEviiiiPKiS2_PKdS4_diPdS5_S5_S5_PiS2_S5_i"
    assert _run(_remarks(pcg, 128, 96)).returncode == 1
