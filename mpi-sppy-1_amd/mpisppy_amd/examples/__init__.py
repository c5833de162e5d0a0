"""Example scenario models (farmer, aircond)."""
