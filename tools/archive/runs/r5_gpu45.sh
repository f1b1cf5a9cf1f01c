#!/bin/bash
# round 5: Q bisect + C5 trace, then the boot-bwd A/B
bash tools/archive/runs/r5_gpu4.sh && bash tools/archive/runs/r5_gpu5.sh
