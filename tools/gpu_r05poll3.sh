#!/bin/bash
# The done word stored relaxed after an agent-scope fence (in-tree) against a system-scope
# release store (lib_pollrel) and the completion event (lib_evbase); config 3, interleaved.
set -e
bash tools/ab.sh 100 "- tools/variants/lib_pollrel.so tools/variants/lib_evbase.so - tools/variants/lib_pollrel.so tools/variants/lib_evbase.so"
