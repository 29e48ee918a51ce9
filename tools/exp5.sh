#!/bin/bash
timeout -k 10 300 python tools/dstamps.py || exit $?
LZ4E_COMPRESS_LDS_MAX=0 timeout -k 10 300 python tools/stamps.py || exit $?
