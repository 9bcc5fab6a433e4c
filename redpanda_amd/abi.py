"""numpy mirrors of the C-ABI data layouts declared in include/rpgpu.h.

These are layouts only (no logic): the product wrapper (`redpanda_amd._lib`),
the tests and the oracle wrapper all view device/host result buffers through
them, so parity checks are plain array comparisons.
"""
import numpy as np

HEADER_SIZE = 61

CODEC_NONE, CODEC_GZIP, CODEC_SNAPPY, CODEC_LZ4, CODEC_ZSTD = 0, 1, 2, 3, 4
# rpgpu_status
OK, E_INVALID, E_NO_DEVICE, E_NOMEM, E_OVERFLOW, E_CODEC, E_UNSUPPORTED, E_HIP = 0, -1, -2, -3, -4, -5, -6, -7
PENDING = 1
# rpgpu_stamp flags
STAMP_OFFSETS, STAMP_CRC = 1, 2

ERRC_NONE = 0
ERRC_END_OF_STREAM = 1
ERRC_HEADER_ONLY_CRC_MISSMATCH = 2
ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES = 3
ERRC_FALLOCATED_FILE_READ_ZERO_BYTES_FOR_HEADER = 4
ERRC_NOT_ENOUGH_BYTES_IN_PARSER_FOR_ONE_RECORD = 5

F_HEADER_OK = 1 << 0
F_COMPLETE = 1 << 1
F_CRC_OK = 1 << 2
F_COMPRESSED = 1 << 3
F_CODEC_INVALID = 1 << 4
F_CODEC_UNSUPPORTED = 1 << 5
F_CODEC_OK = 1 << 6
F_PARSED = 1 << 7
F_PARSE_ASYNC_OK = 1 << 8
F_PARSE_OK = 1 << 9
F_INDEX_WRITTEN = 1 << 10
F_WIRE_V2 = 1 << 11
F_DECODE_OVERFLOW = 1 << 12

PARSE_ERR_NONE = 0
PARSE_ERR_ATTR_EOF = 1
PARSE_ERR_COPY_NEGATIVE = 2
PARSE_ERR_HEADER_RESERVE = 3
PARSE_ERR_TRAILING = 4
PARSE_ERR_INDEX_CAPACITY = 5

JOB_CRC = 1 << 0
JOB_PARSE = 1 << 1
JOB_DECODE = 1 << 2
JOB_HOST_CODECS = 1 << 3

LAYOUT_DISK = 0
LAYOUT_WIRE = 1

BATCH_RESULT = np.dtype([
    ("file_pos", "<u8"), ("base_offset", "<i8"), ("first_timestamp", "<i8"),
    ("max_timestamp", "<i8"), ("producer_id", "<i8"), ("size_bytes", "<i4"),
    ("record_count", "<i4"), ("last_offset_delta", "<i4"), ("base_sequence", "<i4"),
    ("header_crc", "<u4"), ("crc", "<u4"), ("crc_computed", "<u4"),
    ("header_crc_computed", "<u4"), ("flags", "<u4"), ("segment", "<u4"),
    ("index_base", "<u8"), ("decoded_off", "<u8"), ("records_parsed", "<u4"),
    ("decoded_len", "<u4"), ("decoded_crc", "<u4"), ("decoded_header_crc", "<u4"),
    ("attrs", "<i2"), ("producer_epoch", "<i2"), ("type", "i1"), ("parse_err", "u1"),
    ("reserved0", "<u2"), ("reserved1", "<u8"),
])
assert BATCH_RESULT.itemsize == 128

RECORD_INDEX = np.dtype([
    ("batch", "<u4"), ("rec_pos", "<u4"), ("ts_delta", "<i8"), ("length", "<i4"),
    ("offset_delta", "<i4"), ("key_len", "<i4"), ("key_pos", "<u4"), ("val_len", "<i4"),
    ("val_pos", "<u4"), ("hdr_count", "<i4"), ("hdr_pos", "<u4"), ("end_pos", "<u4"),
    ("attrs", "i1"), ("pad", "u1", (3,)), ("reserved", "<u4", (2,)),
])
assert RECORD_INDEX.itemsize == 64

SEGMENT_SUMMARY = np.dtype([
    ("first_batch", "<u8"), ("n_batches", "<u8"), ("terminal_pos", "<u8"),
    ("bytes_consumed", "<u8"), ("terminal_errc", "<i4"), ("terminal_eof", "<i4"),
    ("has_checkpoint", "<i4"), ("first_bad", "<u4"), ("ckpt_last_offset", "<i8"),
    ("ckpt_truncate_pos", "<u8"), ("n_records", "<u8"), ("reserved", "<u8", (2,)),
])
assert SEGMENT_SUMMARY.itemsize == 88

# rpgpu_index_state (include/rpgpu.h): index_state header after recovery
INDEX_STATE = np.dtype([
    ("base_offset", "<i8"), ("max_offset", "<i8"), ("base_timestamp", "<i8"),
    ("max_timestamp", "<i8"), ("first_entry", "<u8"), ("n_entries", "<u8"),
    ("assert_batch", "<i8"), ("tracked", "<u8"),
])
assert INDEX_STATE.itemsize == 64
INDEX_DEFAULT_STEP = 32768  # segment_index::default_data_buffer_step (storage/segment_index.h:49)

JOB_TOTALS = np.dtype([
    ("n_batches", "<u8"), ("n_records", "<u8"), ("decoded_bytes", "<u8"),
    ("batch_capacity_needed", "<u8"), ("record_capacity_needed", "<u8"),
    ("decoded_capacity_needed", "<u8"), ("overflow", "<u4"), ("n_rewalks", "<u4"),
    ("reserved", "<u8", (2,)),
])
assert JOB_TOTALS.itemsize == 72

# fields of rpgpu_batch_result that are outputs of the engine and compared
# bit-exactly against the oracle (reserved fields excluded)
BATCH_COMPARE_FIELDS = [n for n in BATCH_RESULT.names if not n.startswith("reserved")]
RECORD_COMPARE_FIELDS = [n for n in RECORD_INDEX.names if n not in ("pad", "reserved")]
SUMMARY_COMPARE_FIELDS = [n for n in SEGMENT_SUMMARY.names if n != "reserved"]
