"""CPU: the host mirror's config handling (AggregationConfig.transform -> UnifiedConfig,
config.rs:252-335) and the flushed-row layout (no device needed)."""
from netgauze_amd import _lib
from netgauze_amd.aggregate import unify


def test_unify_keeps_transform_order_and_indices():
    transform = {(0, 8): "Key", (0, 1): {0: "Add", 1: "Max"}, (0, 12): {1: "Key"}, (0, 6): "BoolMapOr"}
    assert unify(transform) == [(0, 8, 0, _lib.NGZ_AGG_KEY), (0, 1, 0, _lib.NGZ_AGG_ADD),
                                (0, 1, 1, _lib.NGZ_AGG_MAX), (0, 12, 1, _lib.NGZ_AGG_KEY),
                                (0, 6, 0, _lib.NGZ_AGG_OR)]


def test_row_dtype_matches_header():
    assert _lib.AGG_ROW_DTYPE.itemsize == 88
    assert _lib.AGG_ROW_DTYPE.fields["record_count"][1] == 16
    assert _lib.AGG_ROW_DTYPE.fields["template_bits"][1] == 56
    assert _lib.AGG_ROW_DTYPE.fields["domain_bits"][1] == 72
