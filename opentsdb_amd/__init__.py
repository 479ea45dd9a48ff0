"""opentsdb_amd — MI355X-native query-time aggregation for OpenTSDB 1.1.

The hot path (RowSeq decode -> Span downsample -> SpanGroup lerp/rate merge ->
Aggregators) runs as hand-written HIP kernels for gfx950 inside
libtsdbhip.so (opentsdb_amd/csrc). This package is the host-side mirror of the
reference's call surface (Aggregators, SpanGroup/DataPoints, CompactionQueue)
over that C-ABI.
"""
__all__ = ["_abi", "packing", "synth"]
