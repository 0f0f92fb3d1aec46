"""Filesystem locations of the in-tree native libraries."""
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # mqtt-server_amd/
LIB_DIR = os.path.join(PKG_DIR, "lib")
REPO_DIR = os.path.dirname(PKG_DIR)
