#!/bin/bash
# A/B + update/merge parity (gpu_abp.sh), then the EAP parity tests
set -u
bash scripts/gpu_abp.sh ${1:-abe} ${2:-3} || exit $?
bash scripts/gpu_eap_parity.sh ${1:-abe}_eap
