"""Drop-in for the reference's compiled decoder modules (setup.py:26-86): the same
module and function names, backed by the HIP decoder (ccmi_decode_file)."""
