FROM registry.access.redhat.com/ubi8/ubi-minimal:8.3-201
RUN microdnf update && microdnf install -y php && microdnf clean all
WORKDIR /app
COPY . .
EXPOSE 8080
CMD ["php", "-S", "0.0.0.0:8080"]
