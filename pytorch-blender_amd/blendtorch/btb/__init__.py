"""(filled in below)"""
