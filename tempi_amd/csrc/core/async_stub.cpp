// temporary: transport / async subsystems not yet built
namespace tempi {
void async_init() {}
void async_finalize() {}
void transport_init() {}
void transport_finalize() {}
} // namespace tempi
