"""grayscott_amd.models"""
