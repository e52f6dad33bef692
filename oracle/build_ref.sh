#!/bin/bash
# Compile the reference's own NFCore property/record classes and NFCScheduleModule
# from /root/reference (read-only) together with oracle/ref_harness.cpp into
# oracle/_ref/nf_ref_harness.  No reference source is copied into this repo.
set -euo pipefail
cd "$(dirname "$0")"
REF=${REF:-/root/reference}
if [ ! -d "$REF/NFComm" ]; then
  echo "reference tree not present ($REF); using prebuilt _ref/ if any" >&2
  exit 0
fi
make -s ref REF="$REF"
