"""Filesystem locations of the in-tree native libraries."""
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # mqtt-server_amd/
# (MQ_LIB_DIR: a development build of the same library, e.g. lib_dev/ from `make DEV=1`, for A/B runs)
LIB_DIR = os.environ.get("MQ_LIB_DIR") or os.path.join(PKG_DIR, "lib")
REPO_DIR = os.path.dirname(PKG_DIR)
