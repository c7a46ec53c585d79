#!/bin/bash
# ba.py's launcher (Generals_Byzantine_program.sh:1) for the libba_hip front end:
#   ./generals.sh N [--seed S] [--om M]
cd "$(dirname "$0")" && exec python3 -m ba_amd.repl "$@"
