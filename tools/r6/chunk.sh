#!/bin/bash
# round 6: backward XCD chunk 16 (cur4) vs 32 / 64 consecutive tiles per XCD
TAG=chunk VARIANTS="cur4 ch32 ch64" LEGS="micro b4096 poac" ROUNDS=2 bash tools/r6/ab_libs.sh
