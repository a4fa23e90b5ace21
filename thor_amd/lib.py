"""ctypes binding of libthor_amd.so (the C-ABI in include/thor_amd.h and
include/thor_kernels.h).  The library is the product; there is no CPU
fallback: if it is missing or no GPU is present, calls fail loudly."""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("THOR_AMD_LIB") or os.path.join(HERE, "libthor_amd.so")

_lib = None


class ThorSeq(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("bipred", C.c_int32), ("deblocking", C.c_int32),
                ("clpf", C.c_int32), ("tb_split_enable", C.c_int32), ("interp_ref", C.c_int32)]


class ThorFrameHdr(C.Structure):
    _fields_ = [("frame_num", C.c_int32), ("frame_type", C.c_int32), ("qp", C.c_int32), ("clpf_on", C.c_int32),
                ("interp_ref", C.c_int32 * 2), ("interp_ratio", C.c_int32), ("interp_pos", C.c_int32)]


class ThorYuvPlanes(C.Structure):
    _fields_ = [("y", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p), ("stride_y", C.c_int32),
                ("stride_c", C.c_int32)]


class ThorEncParams(C.Structure):
    """thor_enc_params_t (include/thor_amd.h) = enc_params (enc/mainenc.h:34-88)."""
    _fields_ = [(n, C.c_int32) for n in ("width", "height", "qp", "num_frames", "skip")] + \
        [(n, C.c_float) for n in ("frame_rate", "lambda_coeffI", "lambda_coeffP", "lambda_coeffB", "lambda_coeffB0",
                                  "lambda_coeffB1", "lambda_coeffB2", "lambda_coeffB3", "early_skip_thr")] + \
        [(n, C.c_int32) for n in ("enable_tb_split", "enable_pb_split", "max_num_ref", "HQperiod", "num_reorder_pics",
                                  "dyadic_coding", "interp_ref", "dqpP", "dqpB", "dqpB0", "dqpB1", "dqpB2", "dqpB3")] + \
        [(n, C.c_float) for n in ("mqpP", "mqpB", "mqpB0", "mqpB1", "mqpB2", "mqpB3")] + \
        [(n, C.c_int32) for n in ("dqpI", "intra_period", "intra_rdo", "rdoq", "max_delta_qp", "delta_qp_step",
                                  "encoder_speed", "sync", "deblocking", "clpf", "snrcalc", "use_block_contexts",
                                  "enable_bipred")]


class ThorFrameIn(C.Structure):
    _fields_ = [("blocks", C.c_void_p), ("nblocks", C.c_int32), ("coeffs", C.c_void_p), ("clpf_flags", C.c_void_p),
                ("intra_list", C.c_void_p), ("n_intra", C.c_int32), ("tu_list", C.c_void_p), ("n_tu", C.c_int32),
                ("clpf_list", C.c_void_p), ("n_clpf", C.c_int32), ("slow_list", C.c_void_p), ("n_slow", C.c_int32)]


class ThorFrameImage(C.Structure):
    """thor_frame_image_t (include/thor_amd.h)."""
    _fields_ = [(n, C.c_uint64) for n in ("bytes", "off_blocks", "off_coeffs", "off_flags", "off_intra", "off_tus",
                                          "off_clpf", "off_slow")] + \
        [(n, C.c_int32) for n in ("nblocks", "ncoeffs", "n_flags", "n_intra", "n_tu", "n_clpf", "n_slow")]


class ThorParsedFrame(C.Structure):
    """thor_parsed_frame_t (include/thor_amd.h)."""
    _fields_ = [("seq", ThorSeq), ("hdr", ThorFrameHdr), ("decode_order", C.c_int32), ("num_ref", C.c_int32),
                ("blocks", C.c_void_p), ("nblocks", C.c_int32), ("coeffs", C.c_void_p), ("ncoeffs", C.c_int32),
                ("clpf_flags", C.c_void_p), ("nclpf", C.c_int32)]


# Every symbol the public headers declare (checked by tests/test_capi.py).
BATCHED_SYMBOLS = [
    "thor_dec_create", "thor_dec_destroy", "thor_dec_frame", "thor_dec_frames", "thor_dec_frame_begin",
    "thor_dec_frame_end", "thor_dec_set_band", "thor_dec_set_band_local", "thor_dec_frame_finish", "thor_dec_set_band_intra", "thor_dec_set_band_pad", "thor_dec_frame_intra", "thor_dec_get_rows", "thor_dec_put_rows", "thor_dec_put_ref_rows", "thor_dec_pad_frame", "thor_build_intra_list", "thor_build_tu_list", "thor_build_clpf_list", "thor_build_slow_list", "thor_dec_set_stop_stage",
    "thor_dec_read_frame", "thor_dec_write_frame", "thor_dec_set_timing", "thor_dec_stage_ms", "thor_dec_stage_marks", "thor_dec_sync", "thor_dec_stream", "thor_dec_set_stream",
    "thor_enc_tu_batch", "thor_enc_cost_batch",
    "thor_enc_default_params", "thor_enc_check_params", "thor_enc_create", "thor_enc_destroy", "thor_enc_num_frames",
    "thor_enc_next_input", "thor_enc_stream", "thor_enc_set_cu_mask", "thor_enc_frames", "thor_enc_frames_begin", "thor_enc_frames_end", "thor_enc_frame", "thor_enc_frame_bytes",
    "thor_enc_plan_input", "thor_enc_seq_begin", "thor_enc_seq_ready", "thor_enc_seq_chunk", "thor_enc_seq_end", "thor_enc_seq_profile", "thor_enc_rows_profile",
    "thor_enc_read_recon", "thor_enc_reset", "thor_enc_debug_stall", "thor_enc_record_sb_costs", "thor_enc_sb_costs",
    "thor_parser_create", "thor_parser_destroy", "thor_parser_seq", "thor_parse_frame", "thor_frame_image",
    "thor_ti_create", "thor_ti_destroy", "thor_interpolate_frames", "thor_ti_read_fields", "thor_ti_status",
    "thor_dev_alloc", "thor_dev_free", "thor_h2d", "thor_d2h", "thor_device_count", "thor_version",
    "thor_last_create_error",
]
L2_SURFACE_SYMBOLS = ["deblock_frame_y", "deblock_frame_uv", "make_top_and_left", "get_intra_prediction", "dequantize",
                      "reconstruct_block", "quantize"]
SIMD_SURFACE_SYMBOLS = [
    "block_avg_simd", "sad_calc_simd_unaligned", "get_inter_prediction_luma_simd", "get_inter_prediction_chroma_simd",
    "transform_simd", "inverse_transform_simd", "clpf_block4", "clpf_block8",
    "sad_calc_simd", "ssd_calc_simd", "widesad_calc_simd", "detect_clpf_simd", "sad_calc_fasthalf_simd",
    "sad_calc_fastquarter_simd",
]


def load(path: str = LIB_PATH):
    """Load the library (building it first if this checkout can)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        try:
            from . import build as _b

            _b.build()
        except Exception as e:  # pragma: no cover - depends on toolchain
            raise RuntimeError("libthor_amd.so is missing and could not be built: %s" % e) from e
    L = C.CDLL(path)
    P, i = C.c_void_p, C.c_int
    L.thor_version.restype = C.c_char_p
    L.thor_device_count.restype = i
    L.thor_dec_create.argtypes = [C.POINTER(ThorSeq), i, i]
    L.thor_dec_create.restype = P
    L.thor_dec_destroy.argtypes = [P]
    L.thor_dec_frame.argtypes = [P, C.POINTER(ThorFrameHdr), P, i, P, P, P, i, P, i]
    L.thor_dec_frame.restype = i
    L.thor_dec_frames.argtypes = [P, i, P, P]
    L.thor_dec_frames.restype = i
    L.thor_dec_frame_begin.argtypes = [P, P, P]
    L.thor_dec_frame_begin.restype = i
    L.thor_dec_frame_end.argtypes = [P]
    L.thor_dec_frame_end.restype = i
    L.thor_dec_set_band.argtypes = [P, i, i]
    L.thor_dec_set_band.restype = i
    L.thor_dec_set_band_local.argtypes = [P, i]
    L.thor_dec_set_band_local.restype = i
    L.thor_dec_set_band_intra.argtypes = [P, i]
    L.thor_dec_set_band_intra.restype = i
    L.thor_dec_set_band_pad.argtypes = [P, i]
    L.thor_dec_set_band_pad.restype = i
    L.thor_dec_frame_intra.argtypes = [P]
    L.thor_dec_frame_intra.restype = i
    L.thor_dec_frame_finish.argtypes = [P]
    L.thor_dec_frame_finish.restype = i
    L.thor_dec_get_rows.argtypes = [P, i, i, i, P]
    L.thor_dec_get_rows.restype = i
    L.thor_dec_put_rows.argtypes = [P, i, i, i, P]
    L.thor_dec_put_rows.restype = i
    L.thor_dec_put_ref_rows.argtypes = [P, i, i, i, P]
    L.thor_dec_put_ref_rows.restype = i
    L.thor_dec_pad_frame.argtypes = [P, i]
    L.thor_dec_pad_frame.restype = i
    L.thor_build_intra_list.argtypes = [P, i, P]
    L.thor_build_intra_list.restype = i
    L.thor_build_tu_list.argtypes = [P, i, P]
    L.thor_build_tu_list.restype = i
    L.thor_build_clpf_list.argtypes = [P, i, P]
    L.thor_build_clpf_list.restype = i
    L.thor_build_slow_list.argtypes = [P, i, i, i, P]
    L.thor_build_slow_list.restype = i
    L.thor_dec_set_stop_stage.argtypes = [P, i]
    L.thor_dec_read_frame.argtypes = [P, i, P, P, P]
    L.thor_dec_read_frame.restype = i
    L.thor_dec_write_frame.argtypes = [P, i, P, P, P]
    L.thor_dec_write_frame.restype = i
    L.thor_dec_sync.argtypes = [P]
    L.thor_dec_sync.restype = i
    L.thor_dec_stream.argtypes = [P]
    L.thor_dec_stream.restype = P
    L.thor_dec_set_stream.argtypes = [P, P]
    L.thor_dec_set_timing.argtypes = [P, i]
    L.thor_dec_stage_ms.argtypes = [P, C.POINTER(C.c_double), i]
    L.thor_dec_stage_ms.restype = i
    L.thor_dec_stage_marks.argtypes = [P, P, P, i]
    L.thor_dec_stage_marks.restype = i
    L.thor_enc_tu_batch.argtypes = [P, i, P, P, P, P, P, P, P]
    L.thor_enc_tu_batch.restype = i
    L.thor_enc_cost_batch.argtypes = [P, P, P, P, C.c_double, P, i, P]
    L.thor_enc_cost_batch.restype = i
    EP = C.POINTER(ThorEncParams)
    L.thor_enc_default_params.argtypes = [EP]
    L.thor_enc_check_params.argtypes = [EP]
    L.thor_enc_check_params.restype = i
    L.thor_enc_create.argtypes = [EP, i]
    L.thor_enc_create.restype = P
    L.thor_enc_destroy.argtypes = [P]
    L.thor_enc_num_frames.argtypes = [P]
    L.thor_enc_num_frames.restype = i
    L.thor_enc_next_input.argtypes = [P]
    L.thor_enc_next_input.restype = i
    L.thor_enc_reset.argtypes = [P]
    L.thor_enc_reset.restype = i
    L.thor_enc_debug_stall.argtypes = [i, i]
    L.thor_enc_debug_stall.restype = i
    L.thor_enc_stream.argtypes = [P]
    L.thor_enc_stream.restype = P
    L.thor_enc_set_cu_mask.argtypes = [P, C.POINTER(C.c_uint32), i]
    L.thor_enc_set_cu_mask.restype = i
    L.thor_enc_frames.argtypes = [P, i, P, P]
    L.thor_enc_frames.restype = i
    L.thor_enc_frames_begin.argtypes = [P, i, P, P]
    L.thor_enc_frames_begin.restype = i
    L.thor_enc_frames_end.argtypes = [P, i]
    L.thor_enc_frames_end.restype = i
    L.thor_enc_frame.argtypes = [P, P, i]
    L.thor_enc_frame.restype = i
    L.thor_enc_frame_bytes.argtypes = [P, P, C.c_size_t]
    L.thor_enc_frame_bytes.restype = C.c_longlong
    L.thor_enc_plan_input.argtypes = [P, i]
    L.thor_enc_plan_input.restype = i
    L.thor_enc_seq_begin.argtypes = [P, i, i, P, P, i, C.c_longlong]
    L.thor_enc_seq_begin.restype = i
    L.thor_enc_seq_ready.argtypes = [P, P, i]
    L.thor_enc_seq_ready.restype = i
    L.thor_enc_seq_chunk.argtypes = [P, i, i, P, C.c_size_t]
    L.thor_enc_seq_chunk.restype = C.c_longlong
    L.thor_enc_rows_profile.argtypes = [i, P]
    L.thor_enc_rows_profile.restype = i
    L.thor_enc_seq_profile.argtypes = [P, P, i]
    L.thor_enc_seq_profile.restype = i
    L.thor_enc_seq_end.argtypes = [P, P]
    L.thor_enc_seq_end.restype = i
    L.thor_enc_read_recon.argtypes = [P, P, P, P]
    L.thor_enc_read_recon.restype = i
    L.thor_enc_record_sb_costs.argtypes = [P, i]
    L.thor_enc_record_sb_costs.restype = i
    L.thor_enc_sb_costs.argtypes = [P, P, C.c_size_t, C.POINTER(C.c_int)]
    L.thor_enc_sb_costs.restype = C.c_longlong
    L.thor_parser_create.restype = P
    L.thor_parser_destroy.argtypes = [P]
    L.thor_parser_seq.argtypes = [P, C.POINTER(ThorSeq)]
    L.thor_parser_seq.restype = i
    L.thor_parse_frame.argtypes = [P, P, C.c_size_t, C.POINTER(ThorParsedFrame)]
    L.thor_parse_frame.restype = i
    L.thor_frame_image.argtypes = [C.POINTER(ThorParsedFrame), P, C.c_size_t, C.POINTER(ThorFrameImage)]
    L.thor_frame_image.restype = i
    L.thor_pyramid_levels.argtypes = [i, i]
    L.thor_pyramid_levels.restype = i
    L.thor_scale_pyramid.argtypes = [P, i, i, i, P, P, i, P]
    L.thor_scale_pyramid.restype = i
    L.thor_scale_pyramid2.argtypes = [P, P, i, i, i, P, P, P, i, P]
    L.thor_scale_pyramid2.restype = i
    L.thor_interp_comp.argtypes = [P, i, P, i, P, i, P, P] + [i] * 9 + [P]
    L.thor_interp_comp.restype = i
    L.thor_interp_frame.argtypes = [P, P, P, i, i, i, i, i, i, P]
    L.thor_interp_frame.restype = i
    L.thor_ti_create.argtypes = [i, i, i]
    L.thor_ti_create.restype = P
    L.thor_ti_destroy.argtypes = [P]
    L.thor_interpolate_frames.argtypes = [P, C.POINTER(ThorYuvPlanes), C.POINTER(ThorYuvPlanes), i,
                                          C.POINTER(ThorYuvPlanes), i, i, P]
    L.thor_interpolate_frames.restype = i
    L.thor_ti_read_fields.argtypes = [P, i, P, P]
    L.thor_ti_read_fields.restype = i
    L.thor_ti_status.argtypes = [P]
    L.thor_ti_status.restype = i
    # the reference's SIMD kernel surface (include/thor_kernels.h)
    u8p = P
    L.transform_simd.argtypes = [P, P, i, i]
    L.inverse_transform_simd.argtypes = [P, P, i]
    L.block_avg_simd.argtypes = [P, P, P, i, i, i, i, i]
    L.sad_calc_simd_unaligned.argtypes = [P, P, i, i, i, i]
    L.sad_calc_simd_unaligned.restype = i
    L.sad_calc_simd.argtypes = [P, P, i, i, i, i]
    L.sad_calc_simd.restype = i
    L.ssd_calc_simd.argtypes = [P, P, i, i, i]
    L.ssd_calc_simd.restype = i
    L.widesad_calc_simd.argtypes = [P, P, i, i, i, i, C.POINTER(C.c_int)]
    L.widesad_calc_simd.restype = C.c_uint
    for n in ("sad_calc_fasthalf_simd", "sad_calc_fastquarter_simd"):
        getattr(L, n).argtypes = [P, P, i, i, i, i, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        getattr(L, n).restype = C.c_uint
    L.detect_clpf_simd.argtypes = [P, P, i, i, i, i, i, i, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.clpf_block4.argtypes = [u8p, u8p, i, i, i, i, i, i]
    L.clpf_block8.argtypes = [u8p, u8p, i, i, i, i, i, i]
    L.get_inter_prediction_luma_simd.argtypes = [i, i, i, i, P, i, P, i, i]
    L.get_inter_prediction_chroma_simd.argtypes = [i, i, i, i, P, i, P, i]
    L.thor_dev_alloc.argtypes = [C.c_size_t]
    L.thor_dev_alloc.restype = P
    L.thor_dev_free.argtypes = [P]
    L.thor_h2d.argtypes = [P, P, C.c_size_t]
    L.thor_h2d.restype = i
    L.thor_d2h.argtypes = [P, P, C.c_size_t]
    L.thor_d2h.restype = i
    L.thor_last_create_error.argtypes = [C.POINTER(C.c_size_t), C.c_char_p, C.c_size_t]
    L.thor_last_create_error.restype = i
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError("%s failed with status %d" % (what, rc))


class CreateError(RuntimeError):
    """A thor_*_create returned NULL: `code` (THOR_ERR_ARG / _NOMEM / _HIP),
    `bytes` (THOR_ERR_NOMEM: the allocation that failed) and the library's
    one-line reason."""

    def __init__(self, what: str, code: int, nbytes: int, reason: str):
        super().__init__("%s failed (%s%s): %s" % (what, ERR_NAMES.get(code, str(code)),
                                                   ", %d bytes" % nbytes if code == THOR_ERR_NOMEM else "", reason))
        self.code, self.bytes, self.reason = code, nbytes, reason


THOR_OK, THOR_ERR_ARG, THOR_ERR_HIP, THOR_ERR_NOMEM, THOR_ERR_REF = 0, -1, -2, -3, -4
ERR_NAMES = {THOR_ERR_ARG: "THOR_ERR_ARG", THOR_ERR_HIP: "THOR_ERR_HIP", THOR_ERR_NOMEM: "THOR_ERR_NOMEM",
             THOR_ERR_REF: "THOR_ERR_REF"}


def create_error(what: str) -> CreateError:
    """The reason the calling thread's last create returned NULL."""
    L = load()
    n = C.c_size_t(0)
    buf = C.create_string_buffer(256)
    code = L.thor_last_create_error(C.byref(n), buf, len(buf))
    return CreateError(what, code, n.value, buf.value.decode(errors="replace"))
