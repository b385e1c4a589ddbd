"""grayscott_amd.utils"""
