"""grayscott_amd.ops"""
