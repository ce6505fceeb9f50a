"""pinot_amd — MI355X-native (gfx950 HIP) segment query hot path for Apache Pinot.

Dictionary-encoded forward-index scan, predicate filtering and aggregation / group-by behind a C-ABI
(include/pinot_amd.h, libpinot_amd.so). See DESIGN.md.
"""
from . import query  # noqa: F401
from .query import parse_sql  # noqa: F401
from .segment import Segment, Column, create_segment  # noqa: F401
from ._lib import PinotAmdError, lib  # noqa: F401
