"""The reference's operating points (config_*.txt at the reference root) as
encoder flag dictionaries (data only: the `-flag value` lines of each file,
input / output / size / frame-count lines left to the caller).  Used to drive
the device encoder with exactly the parameters the reference Thorenc reads
(enc/strings.c:64-122 parses these files)."""
from __future__ import annotations

_COMMON_LDB = {"-f": "60", "-qp": "32", "-HQperiod": "12", "-mqpP": "1.2", "-dqpI": "-2",
               "-lambda_coeffI": "0.8", "-lambda_coeffP": "1.2"}

CONFIGS = {
    # config_LDB_low_complexity.txt:19-26
    "config_LDB_low_complexity.txt": dict(_COMMON_LDB, **{
        "-intra_rdo": "0", "-enable_tb_split": "0", "-enable_pb_split": "0", "-early_skip_thr": "1.0",
        "-max_num_ref": "2", "-use_block_contexts": "1", "-enable_bipred": "0", "-encoder_speed": "2"}),
    # config_LDB_medium_complexity.txt:19-26
    "config_LDB_medium_complexity.txt": dict(_COMMON_LDB, **{
        "-intra_rdo": "1", "-enable_tb_split": "0", "-enable_pb_split": "0", "-early_skip_thr": "0.8",
        "-max_num_ref": "2", "-use_block_contexts": "1", "-enable_bipred": "1", "-encoder_speed": "1"}),
    # config_LDB_high_efficiency.txt:20-28
    "config_LDB_high_efficiency.txt": dict(_COMMON_LDB, **{
        "-intra_rdo": "1", "-enable_tb_split": "1", "-enable_pb_split": "1", "-early_skip_thr": "0.3",
        "-max_num_ref": "4", "-use_block_contexts": "1", "-enable_bipred": "1", "-encoder_speed": "0",
        "-max_delta_qp": "1"}),
}

# config_HDB16_*.txt:8-35 (hierarchical B, 16-frame sub-GOP, interpolated references)
_COMMON_HDB16 = {"-f": "60", "-qp": "32", "-HQperiod": "1", "-num_reorder_pics": "15", "-interp_ref": "1",
                 "-dqpI": "-2", "-dqpB0": "2", "-dqpB1": "1", "-dqpB2": "0", "-dqpB3": "0",
                 "-mqpP": "1.2", "-mqpB": "1.2", "-mqpB0": "1.075", "-mqpB1": "1.15", "-mqpB2": "1.225",
                 "-mqpB3": "1.3", "-lambda_coeffI": "0.8", "-lambda_coeffP": "1.2", "-lambda_coeffB": "1.2",
                 "-lambda_coeffB0": "1.2", "-lambda_coeffB1": "1.2", "-lambda_coeffB2": "1.2",
                 "-lambda_coeffB3": "1.2"}
CONFIGS.update({
    # config_HDB16_low_complexity.txt:40-47
    "config_HDB16_low_complexity.txt": dict(_COMMON_HDB16, **{
        "-intra_rdo": "0", "-enable_tb_split": "0", "-enable_pb_split": "0", "-early_skip_thr": "1.0",
        "-max_num_ref": "2", "-use_block_contexts": "1", "-enable_bipred": "1", "-encoder_speed": "2"}),
    # config_HDB16_medium_complexity.txt:40-47
    "config_HDB16_medium_complexity.txt": dict(_COMMON_HDB16, **{
        "-intra_rdo": "1", "-enable_tb_split": "0", "-enable_pb_split": "0", "-early_skip_thr": "0.8",
        "-max_num_ref": "2", "-use_block_contexts": "1", "-enable_bipred": "1", "-encoder_speed": "1"}),
    # config_HDB16_high_efficiency.txt:40-48
    "config_HDB16_high_efficiency.txt": dict(_COMMON_HDB16, **{
        "-intra_rdo": "1", "-enable_tb_split": "1", "-enable_pb_split": "1", "-early_skip_thr": "0.3",
        "-max_num_ref": "4", "-use_block_contexts": "1", "-enable_bipred": "1", "-encoder_speed": "0",
        "-max_delta_qp": "1"}),
})


def flags(config: str, width: int, height: int, frames: int, extra=()) -> list:
    """Command-line flags for `config` (later flags override earlier ones, as
    the reference's parser does)."""
    d = dict(CONFIGS[config])
    d.update({"-width": str(width), "-height": str(height), "-n": str(frames)})
    it = list(extra)
    for k, v in zip(it[0::2], it[1::2]):
        d[k] = v
    out = []
    for k, v in d.items():
        out += [k, v]
    return out
