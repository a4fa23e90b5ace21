"""Host logic: reference-ring sizing from the parsed frame headers
(thor_amd.decoder.ring_slots).  The GPU side (a ring of exactly that many
slots decodes bit-exactly, one fewer reports THOR_ERR_REF) is
tests/test_gpu_streams.py::test_ring_sized_from_stream."""
import os

import pytest

from conftest import GOLD, trace_path
from thor_amd.decoder import MAX_SLOTS, ring_slots
from thor_amd.trace import load_trace

# decode-order reach + 1 of the committed reference streams (low-delay configs reach back to the
# last HQ frame, the HDB16 ones across a sub-GOP): max_num_ref alone does not bound it
EXPECT = {"cif_low": 3, "cif_med": 10, "cif_high": 10, "cif_hdb": 16, "hd_low": 13, "k4_low": 6, "k4_med": 8,
          "w8_low": 4}


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_ring_slots_of_reference_streams(name):
    seq, frames = load_trace(trace_path(name))
    n = ring_slots(frames)
    assert n == EXPECT[name]
    assert seq.max_num_ref + 1 <= n <= MAX_SLOTS
    assert ring_slots(frames, hold=len(frames)) == max(n, len(frames))


def test_ring_slots_counts_interpolation_sources():
    from thor_amd.bitstream import parse_stream

    seq, frames = parse_stream(open(os.path.join(GOLD, "cif_hdbi.bit"), "rb").read())
    assert any(fr.interp_ratio for fr in frames)
    assert ring_slots(frames) == 16


def test_ring_slots_rejects_forward_reference():
    seq, frames = load_trace(trace_path("cif_low"))
    with pytest.raises(ValueError):
        ring_slots(frames[1:])  # frame 1 predicts from frame 0, never decoded


def test_ring_slots_minimum():
    seq, frames = load_trace(trace_path("cif_low"))
    assert ring_slots(frames[:1]) == 2  # an I frame alone: thor_dec_create takes <= 1 as "default"
    assert ring_slots([]) == 2
