#!/bin/bash
# tools/host_crc_bench in each host-CRC form (slice-by-16 tables, 128-bit folding, the widest the CPU
# has), one JSON line per form and length, plus the CPU model.
#   bash tools/host_crc_forms.sh OUT.jsonl
set -o pipefail
out=${1:?usage: host_crc_forms.sh OUT.jsonl}
: > "$out"
echo "{\"cpu\": \"$(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2 | sed 's/^ *//')\"}" >> "$out"
for f in tables pclmul widest; do
  if [ $f = widest ]; then timeout -k 10 120 tools/host_crc_bench >> "$out" || exit 1
  else NSTACK_FCS_HOST_CRC=$f timeout -k 10 120 tools/host_crc_bench >> "$out" || exit 1; fi
done
echo "wrote $(wc -l < "$out") lines to $out"
