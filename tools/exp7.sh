#!/bin/bash
export LZ4E_COMPRESS_LDS_MAX=0
echo "== with stores"; timeout -k 10 300 python tools/stamps.py 2>&1 | grep -E "^==|class (text|ints|records)"
echo "== no stores"; LZ4E_LIB=exp/liblz4e_nostore.so timeout -k 10 300 python tools/stamps.py 2>&1 | grep -E "^==|class (text|ints|records)"
