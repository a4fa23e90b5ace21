"""Create failures say why (thor_last_create_error): unsupported parameters are
THOR_ERR_ARG, exhausted HBM is THOR_ERR_NOMEM with the size of the allocation
that failed (a 320-stream run died on a bare
"thor_dec_create failed")."""
import ctypes as C

import pytest

from thor_amd import lib as L


def _dec_create(width, height, slots=34, device=0):
    lib = L.load()
    cs = L.ThorSeq(width, height, 0, 1, 1, 0, 0)
    return lib.thor_dec_create(C.byref(cs), device, slots)


def test_bad_size_is_arg_error_with_reason():
    """Rejected before any HIP call, so it runs without a GPU."""
    assert not _dec_create(1922, 1080)  # not a multiple of 8 (enc/strings.c:437)
    err = L.create_error("thor_dec_create")
    assert err.code == L.THOR_ERR_ARG
    assert "multiples of 8" in err.reason
    lib = L.load()
    assert not lib.thor_ti_create(0, 64, 0)
    assert L.create_error("thor_ti_create").code == L.THOR_ERR_ARG


@pytest.mark.gpu
def test_ring_over_descriptor_range_is_arg_error():
    """A ring k_recon's 32-bit buffer offsets cannot address."""
    assert not _dec_create(16384, 16384, slots=34)
    err = L.create_error("thor_dec_create")
    assert err.code == L.THOR_ERR_ARG and "2 GiB" in err.reason and err.bytes > 2 ** 31


@pytest.mark.gpu
def test_exhausted_hbm_is_nomem_with_bytes():
    """Take every byte of HBM the library's HIP runtime will hand out (8 GiB,
    then 256 MiB chunks), then ask for a 4K decoder (a 34-slot ring is 483 MB):
    THOR_ERR_NOMEM naming the ring and its size; once the memory is released
    the same create succeeds.  (No torch here: torch's own HIP runtime must not
    be initialised after the library's in this process.)"""
    from thor_amd.decoder import GpuDecoder
    from thor_amd.trace import SeqParams

    lib = L.load()
    held = []
    try:
        for chunk in (8 << 30, 256 << 20):
            while len(held) < 4096:
                p = lib.thor_dev_alloc(chunk)
                if not p:
                    break
                held.append(p)
        seq = SeqParams(3840, 2160, 0, 1, 4, 0, 0, 1, 1, 1, 0)
        with pytest.raises(L.CreateError) as ei:
            GpuDecoder(seq, device=0, slots=34)
        assert ei.value.code == L.THOR_ERR_NOMEM, str(ei.value)
        assert "reference ring" in ei.value.reason
        assert ei.value.bytes >= 34 * 3840 * 2160 * 3 // 2
    finally:
        for p in held:
            lib.thor_dev_free(p)
    d = GpuDecoder(seq, device=0, slots=34)
    d.close()
    assert L.create_error("thor_dec_create").code == L.THOR_OK
