"""Mirror of the reference package of the same name."""
