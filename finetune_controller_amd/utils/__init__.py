"""Shared utilities (metrics CSV, logging, native runtime bindings)."""
