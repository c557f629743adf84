#!/bin/bash
# Rebuilds tests/golden/output_golden.json with the image's conda Qt 5.9.7
# (test infrastructure; run in the build container, never on the GPU box).
# Qt's libraries are reached through a private symlink directory: conda's
# older libstdc++ must not be put on the search path.
set -eo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
T=$(mktemp -d)
QT=/opt/conda/include/qt
mkdir -p $T/qtlib
ln -s /opt/conda/lib/libQt5Core.so.5 /opt/conda/lib/libicu*.so.58 /opt/conda/lib/libz.so.1 $T/qtlib/
python3 $HERE/make_output_items.py
g++ -O1 -std=c++11 -fPIC -DQT_CORE_LIB -I$QT -I$QT/QtCore -o $T/gen $HERE/make_output_golden.cpp \
    /opt/conda/lib/libQt5Core.so.5 -Wl,-rpath,$T/qtlib -Wl,--allow-shlib-undefined
$T/gen $HERE/output_items.json $HERE/output_golden.json
rm -rf $T
echo wrote $HERE/output_golden.json
