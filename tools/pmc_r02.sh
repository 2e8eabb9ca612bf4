#!/bin/bash
# Round-2 PMC sessions: C4 (dragon 1080p), C3 (dragon 960x540), the fill view.
set -u
tools/pmc_all.sh r02pmc_c4 dragon_1920x1080_m0_n1 "k_trace_kd3<16" && \
tools/pmc_all.sh r02pmc_c3 dragon_960x540_m0_n1 "k_trace_kd3<8" --width 960 --height 540 && \
tools/pmc_all.sh r02pmc_fill dragon_1920x1080_m0_n1_fill "k_trace_kd3<16" --view fill
