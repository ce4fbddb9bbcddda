FROM registry.access.redhat.com/ubi8/nodejs-12
ADD . .
RUN npm install
EXPOSE 8080
CMD npm run -d start
