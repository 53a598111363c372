"""Replica-per-GPU mode (C5) through the HIP engine: W processes share
cuda:0, each stepping only the replicas it owns with libdragonboat_amd.so
(rbe_step + rbe_xchg_pack/unpack), exchanging records over gloo staged
through host memory.  Bar: every owned replica equals the oracle stepping
all replicas in one process (test_replica_gloo.run_case)."""
import pytest

from test_replica_gloo import run_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["C2_w2", "C4_w3", "N5_w4", "N7_w3", "C3_iso_w2", "C3_iso_w4", "C2_w4c",
                                  "C3_iso_w4c"])
def test_gpu_replica_per_rank_matches_oracle(gpu_available, name):
    run_case(name, gpu=True)


def test_gpu_replica_per_rank_untraced(gpu_available):
    run_case("C4_w3", gpu=True, trace=False)


def test_gpu_replica_fixed_exchange(gpu_available):
    """The fixed-capacity exchange on the HIP engine (pack and unpack enqueued
    without reading counts back; gloo staging in this one-GPU rehearsal)."""
    run_case("C2_w2", gpu=True, fixed=True)
